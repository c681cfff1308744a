"""The scene-specialised shadow kernel (fast_ray_tracer_amd/csrc/frt_jit.hip).

CPU: every golden scene's generated kernel compiles with hiprtc for gfx950 (the
same generator and options frt_scene_upload uses), and the scenes expected to
be eligible are. GPU: the specialised kernel and the generic walk give
bit-identical canvases, and the specialised one is the one that ran.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_scene

SCENES = sorted(f[:-2] for f in os.listdir(os.path.join(GOLDEN, "scenes")) if f.endswith(".c"))
# scenes whose tree the generator must accept (CSG units of sorted leaves, <= 512 nodes)
ELIGIBLE = {"cornell_direct_800_4x4", "cornell_direct_64_4x4", "checkered_sphere_200", "reflect_refract_160x80",
            "reflect_refract_test_150", "shadow_glamour_150x60", "test_scene_120", "cornell_gi_24"}


@pytest.mark.parametrize("name", SCENES)
def test_jit_source_compiles(built, name):
    from fast_ray_tracer_amd.runtime import jit_check
    rc, log, src = jit_check(load_scene(name))
    assert rc != -1, log[-4000:]
    if name in ELIGIBLE:
        assert rc == 0, log
        assert "frt_jit_shadow" in src
    else:
        assert rc in (0, 1)


def _render(name, jit, **kw):
    from fast_ray_tracer_amd.runtime import GpuRenderer
    old = os.environ.get("FRT_JIT")
    os.environ["FRT_JIT"] = "1" if jit else "0"
    try:
        r = GpuRenderer(load_scene(name))
    finally:
        if old is None:
            del os.environ["FRT_JIT"]
        else:
            os.environ["FRT_JIT"] = old
    try:
        return r.render(stats=True, **kw)
    finally:
        r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell_direct_64_4x4", "reflect_refract_test_150", "shadow_glamour_150x60",
                                  "group_test_150x50", "test_scene_120", "cornell_shipped_48_4x4"])
def test_jit_equals_generic_walk(built, name):
    img_j, st_j = _render(name, True)
    img_g, st_g = _render(name, False)
    assert st_g.shadow_jit == 0
    if name in ELIGIBLE:
        assert st_j.shadow_jit == 1
    assert np.array_equal(img_j, img_g)


@pytest.mark.gpu
def test_jit_equals_generic_walk_on_benchmark_rows(built):
    """cornell 800x800x16: a band of rows through both shadow kernels, bit for bit."""
    img_j, st_j = _render("cornell_direct_800_4x4", True, row_begin=300, row_end=340)
    img_g, _ = _render("cornell_direct_800_4x4", False, row_begin=300, row_end=340)
    assert st_j.shadow_jit == 1
    assert np.array_equal(img_j, img_g)
