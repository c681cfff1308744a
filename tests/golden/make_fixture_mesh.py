#!/usr/bin/env python3
"""Write the textured-mesh fixture (a small stand-in for the missing sibenik.obj).

The reference's sibenik scene (BASELINE cfg4) is an OBJ+MTL cathedral whose
materials carry map_Ka / map_Kd PNG textures and map_bump maps
(scenes/sibenik/sibenik.mtl); sibenik.obj itself is absent from the mount. This
script writes a nave of the same kind, from plain geometry: a floor and two
walls of textured quads (vt coordinates tiled over several texture periods), a
bump-mapped floor, and four columns of smooth triangles (vn) with textures —
every branch of the reference OBJ/MTL path the drop-in must reproduce:
parse_mtl (obj_loader.c:140), parse_map -> read_png + uv_texture +
texture_map_pattern(TRIANGLE_UV_MAP) (obj_loader.c:55-97), fan_triangulation
with v/vt/vn faces (obj_loader.c:220-310), triangle_uv_map (pattern.c:393-440)
and the bump path of prepare_computations.

The textures are the reference's own sibenik PNGs (scene data), copied by
make_golden.py into tests/golden/assets/scenes/sibenik/.

  python tests/golden/make_fixture_mesh.py   # writes tests/golden/assets/scenes/frt_nave/nave.{obj,mtl}
"""
import math
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "assets", "scenes", "frt_nave")

MTL = """# frt fixture: materials of the nave stand-in (textures = the reference's sibenik PNGs)
newmtl floor
    Ka 0.2 0.2 0.2
    Kd 0.8 0.8 0.8
    Ks 0.1 0.1 0.1
    Ns 20
    illum 2
    map_Ka scenes/sibenik/mramor6x6.png
    map_Kd scenes/sibenik/mramor6x6.png
    map_bump scenes/sibenik/mramor6x6-bump.png

newmtl wall
    Ka 0.15 0.15 0.15
    Kd 0.7 0.7 0.7
    Ks 0.0 0.0 0.0
    Ns 10
    illum 2
    map_Kd scenes/sibenik/KAMEN-stup.png

newmtl column
    Ka 0.1 0.1 0.1
    Kd 0.75 0.7 0.6
    Ks 0.3 0.3 0.3
    Ns 60
    illum 2
    map_Kd scenes/sibenik/kamen.png

newmtl brass
    Ka 0.05 0.04 0.02
    Kd 0.4 0.3 0.1
    Ks 0.6 0.5 0.3
    Ns 200
    illum 3
"""


def main():
    os.makedirs(OUT, exist_ok=True)
    v, vt, vn, lines = [], [], [], []

    def vert(x, y, z):
        v.append((x, y, z))
        return len(v)

    def tex(s, t):
        vt.append((s, t))
        return len(vt)

    def nrm(x, y, z):
        vn.append((x, y, z))
        return len(vn)

    def quad_grid(origin, du, dv, nu, nv, tiles, mtl, group):
        """nu x nv quads spanning origin + [0,1]du + [0,1]dv, texture tiled `tiles` times."""
        lines.append("g " + group)
        lines.append("usemtl " + mtl)
        idx = {}
        for j in range(nv + 1):
            for i in range(nu + 1):
                p = [origin[k] + du[k] * i / nu + dv[k] * j / nv for k in range(3)]
                idx[i, j] = (vert(*p), tex(tiles * i / nu, tiles * j / nv))
        for j in range(nv):
            for i in range(nu):
                a, b, c, d = idx[i, j], idx[i + 1, j], idx[i + 1, j + 1], idx[i, j + 1]
                lines.append("f %d/%d %d/%d %d/%d %d/%d" % (a + b + c + d))

    # floor (y = 0), walls at x = +-3, z from -4 to 6
    quad_grid((-3, 0, -4), (6, 0, 0), (0, 0, 10), 6, 10, 3.0, "floor", "floor")
    quad_grid((-3, 0, 6), (0, 0, -10), (0, 4, 0), 10, 4, 2.0, "wall", "wall_left")
    quad_grid((3, 0, -4), (0, 0, 10), (0, 4, 0), 10, 4, 2.0, "wall", "wall_right")

    # four 16-sided columns with smooth normals and wrapped texture
    sides, rings, radius, height = 16, 6, 0.35, 3.5
    for ci, (cx, cz) in enumerate([(-1.6, 0.5), (1.6, 0.5), (-1.6, 3.5), (1.6, 3.5)]):
        lines.append("g column%d" % ci)
        lines.append("usemtl column")
        grid = {}
        for r in range(rings + 1):
            y = height * r / rings
            for s in range(sides + 1):
                a = 2 * math.pi * s / sides
                x, z = math.cos(a), math.sin(a)
                grid[s, r] = (vert(cx + radius * x, y, cz + radius * z), tex(s / sides, 2.0 * r / rings), nrm(x, 0, z))
        for r in range(rings):
            for s in range(sides):
                a, b, c, d = grid[s, r], grid[s + 1, r], grid[s + 1, r + 1], grid[s, r + 1]
                lines.append("f %d/%d/%d %d/%d/%d %d/%d/%d %d/%d/%d" % (a + b + c + d))
    # an untextured faceted brass "lamp" (plain triangles, no vt / vn)
    lines.append("g lamp")
    lines.append("usemtl brass")
    top = vert(0, 2.6, 2.0)
    ring = [vert(0.4 * math.cos(2 * math.pi * k / 8), 2.2, 2.0 + 0.4 * math.sin(2 * math.pi * k / 8)) for k in range(8)]
    bot = vert(0, 1.9, 2.0)
    for k in range(8):
        a, b = ring[k], ring[(k + 1) % 8]
        lines.append("f %d %d %d" % (top, b, a))
        lines.append("f %d %d %d" % (bot, a, b))

    with open(os.path.join(OUT, "nave.obj"), "w") as f:
        f.write("# frt fixture: textured nave (stand-in for the missing sibenik.obj), written by make_fixture_mesh.py\n")
        f.write("mtllib scenes/frt_nave/nave.mtl\n")  # resolved against the working directory, like the reference
        for p in v:
            f.write("v %.6f %.6f %.6f\n" % p)
        for t in vt:
            f.write("vt %.6f %.6f\n" % t)
        for n in vn:
            f.write("vn %.6f %.6f %.6f\n" % n)
        for ln in lines:
            f.write(ln + "\n")
    with open(os.path.join(OUT, "nave.mtl"), "w") as f:
        f.write(MTL)
    print("nave: %d vertices, %d faces" % (len(v), sum(1 for ln in lines if ln.startswith("f "))))


if __name__ == "__main__":
    main()
