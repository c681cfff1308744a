#!/usr/bin/env python3
"""Write the degenerate-mesh fixture: one OBJ group of 600 small triangles, 570 of them packed in [0, 1]
and 30 at x_i = 2 * 17^i (each of the binned SAH's 16 bins holds at most one of those), so the mesh
BVH's build peels one triangle per level
and the tree is deeper than the engine's per-lane mesh stack (frt_engine.hip kMeshStackMax = 32): the
upload must keep the scene (the searches fall back to the group walk where their stack is full) and the
image must equal the plain walk's (tests/test_mesh.py, tests/test_gpu_parity.py).

The scene file tests/golden/scenes/degenerate_mesh_48.c is the reference codegen's main.c layout (as
teapot_low_100.c) with this OBJ, written by this script too.

  python tests/golden/make_fixture_degenerate.py
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OBJ = os.path.join(HERE, "assets", "scenes", "frt_degenerate", "degenerate.obj")
SCENE = os.path.join(HERE, "scenes", "degenerate_mesh_48.c")
N = 600


def main():
    os.makedirs(os.path.dirname(OBJ), exist_ok=True)
    with open(OBJ, "w") as f:
        f.write("# frt fixture: %d triangles, 570 in [0, 1] and 30 at x = 2 * 17^i (a deep SAH tree)\n" % N)
        for i in range(N):
            x = i / 570.0 if i < 570 else 2.0 * 17.0 ** (i - 570)
            y = 0.3 * ((i * 7) % 11 - 5)
            f.write("v %.9f %.9f 0.0\nv %.9f %.9f 0.0\nv %.9f %.9f 0.5\n" % (x, y, x + 0.4, y, x + 0.2, y + 0.4))
        for i in range(N):
            f.write("f %d %d %d\n" % (3 * i + 1, 3 * i + 2, 3 * i + 3))
    src = open(os.path.join(HERE, "scenes", "teapot_low_100.c")).read()
    src = src.replace("scenes/teapot/teapot_low.obj", "scenes/frt_degenerate/degenerate.obj")
    src = src.replace("/tmp/frt_golden/out/teapot_low_100", "/tmp/frt_golden/out/degenerate_mesh_48")
    src = src.replace("camera(100, 100,", "camera(48, 48,")
    src = src.replace("aperture(POINT_APERTURE, 0.4, 1, 1, false, &ap);", "aperture(POINT_APERTURE, 0.0, 1, 1, false, &ap);")
    src = src.replace("global_config.scene.divide_threshold = ", "global_config.scene.divide_threshold = 100000; //")
    assert "degenerate.obj" in src and "camera(48, 48," in src
    with open(SCENE, "w") as f:
        f.write(src)


if __name__ == "__main__":
    main()
