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


def _render(name, jit, beam=True, **kw):
    """Render with the specialised kernels (jit; beam: with the (node, light) pair kernel) or the
    generic walk; the switches are read at upload."""
    from fast_ray_tracer_amd.runtime import GpuRenderer
    env = {"FRT_JIT": "1" if jit else "0", "FRT_JIT_BEAM": "1" if beam else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        r = GpuRenderer(load_scene(name))
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
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


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell_direct_64_4x4", "cornell_shipped_48_4x4", "reflect_refract_test_150",
                                  "test_scene_120", "checkered_sphere_200"])
def test_pair_kernel_equals_per_ray_walk(built, name):
    """frt_jit_beam decides whole (node, light) pairs; the counts it writes must equal what the per-ray
    walk gives for every ray of the pair: the canvas with and without it, bit for bit."""
    img_b, st_b = _render(name, True, beam=True)
    img_r, st_r = _render(name, True, beam=False)
    # the scene-specialised kernels ran (not the generic walk for both)
    assert st_b.shadow_jit == 1 and st_r.shadow_jit == 1
    assert np.array_equal(img_b, img_r)


@pytest.mark.gpu
def test_pair_kernel_on_headline_rows(built):
    """The headline workload (cornell 1920x1080, 8x8 CMJ): row bands through the pair kernel, the
    per-ray kernel alone and the generic walk, bit for bit."""
    for rows in ((200, 208), (640, 648)):
        img_b, st_b = _render("cornell_direct_1920x1080_8x8", True, beam=True, row_begin=rows[0], row_end=rows[1])
        img_r, _ = _render("cornell_direct_1920x1080_8x8", True, beam=False, row_begin=rows[0], row_end=rows[1])
        img_g, _ = _render("cornell_direct_1920x1080_8x8", False, row_begin=rows[0], row_end=rows[1])
        assert st_b.shadow_jit == 1
        assert np.array_equal(img_b, img_r) and np.array_equal(img_b, img_g)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell_direct_64_4x4", "cornell_shipped_48_4x4"])
def test_pair_kernel_batches_split_by_node_range(built, name):
    """The pair kernel's lane index is 32-bit: a batch with more than 2^31 - 1 (node, light part) pairs
    runs as node ranges (frt_engine.hip launch_shadow). FRT_JIT_MAX_PAIRS lowers the limit so a small
    frame takes that path: the canvas must stay bit-identical."""
    img_a, st_a = _render(name, True, beam=True)
    os.environ["FRT_JIT_MAX_PAIRS"] = "4099"
    try:
        img_b, st_b = _render(name, True, beam=True)
    finally:
        del os.environ["FRT_JIT_MAX_PAIRS"]
    assert st_a.shadow_jit == 1 and st_b.shadow_jit == 1
    assert np.array_equal(img_a, img_b)


_ENV_RENDER = r"""
import sys, numpy as np
sys.path.insert(0, {tests!r})
from conftest import load_scene
from fast_ray_tracer_amd.runtime import GpuRenderer
r = GpuRenderer(load_scene({name!r}))
img, st = r.render(stats=True, **{kw!r})
d = st.as_dict()
np.save({out!r}, img)
print("STATS", d["shadow_jit"], d["shadow_tile_pairs"], d["shadow_sub_pairs"])
"""


def _render_env_process(name, env, out, **kw):
    """Render in a fresh process (the tile size and sub-part count are read once per process)."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    penv = dict(os.environ, **{k: v for k, v in env.items() if v is not None})
    for k, v in env.items():  # (None: the variable unset, the engine's own default)
        if v is None:
            penv.pop(k, None)
    p = subprocess.run([sys.executable, "-c", _ENV_RENDER.format(tests=here, name=name, out=str(out), kw=kw)],
                       env=penv, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    stats = [ln.split()[1:] for ln in p.stdout.splitlines() if ln.startswith("STATS")][-1]
    return np.load(str(out)), [int(x) for x in stats]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell_direct_64_4x4", "reflect_refract_test_150", "test_scene_120",
                                  "cornell_shipped_48_4x4"])
def test_tile_and_sub_part_kernels_equal_generic_walk(built, name, tmp_path):
    """The tile pair kernel (frt_jit_tile: runs of consecutive path nodes from their origin box), the sub-part pass
    after it (frt_jit_sub: the tile pairs left mixed, their parts split into sub-parts; 16 single samples of the
    16-sample parts by default, FRT_JIT_SUB=0 off) and frt_jit_beam_list for the nodes of the tile (sub-)pairs left,
    at several tile, part and sub-part sizes, the same-axis slab order (jit::slab_order: tile kernels by default,
    FRT_JIT_ORDER 0 none, 2 every pair kernel) and the tile path split into node ranges (FRT_JIT_MAX_PAIRS: ranges
    start at tile boundaries): each canvas equals the generic walk's bit for bit, and the kernels in question ran."""
    ref, st = _render_env_process(name, {"FRT_JIT": "0"}, tmp_path / "g.npy")
    assert st[0] == 0
    for i, env in enumerate(({"FRT_JIT_TILE": "2"}, {"FRT_JIT_TILE": "32", "FRT_JIT_SUB": "0"},
                             {"FRT_JIT_TILE": "32", "FRT_JIT_ORDER": "0", "FRT_JIT_PART": "17", "FRT_JIT_SUB": "4"},
                             {"FRT_JIT_TILE": "64", "FRT_JIT_ORDER": "2"},
                             {"FRT_JIT_TILE": "8", "FRT_JIT_SUB": "8", "FRT_JIT_MAX_PAIRS": "4099"},
                             # the sub-tile (sub-part) stage's list walked ray by ray without the node pair kernel
                             {"FRT_JIT_NODE_BEAM": "0"}, {"FRT_JIT_NODE_BEAM": "0", "FRT_JIT_SUBTILE": "0"},
                             {"FRT_JIT_NODE_BEAM": "1"}, {"FRT_JIT_SUBTILE_DEEP": "0"},
                             # node-major lanes over the stage's list (groups of 4 / 64 entries; a last group short)
                             {"FRT_JIT_NODE_MAJOR": "4"}, {"FRT_JIT_NODE_MAJOR": "64", "FRT_JIT_SUBTILE": "0"})):
        img, st = _render_env_process(name, env, tmp_path / ("j%d.npy" % i))
        assert st[0] == 1 and st[1] > 0, (env, st)
        if env.get("FRT_JIT_SUB") != "0":
            assert st[2] > 0, (env, st)
        assert np.array_equal(img, ref), env


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell_direct_64_4x4", "checkered_torus_120", "checkered_cylinder_120", "group_test_150x50",
                                  "teapot_low_100", "checkered_sphere_dof_100", "patterns_160x80", "cornell_gi_16",
                                  "test_scene_120", "bump_map_100"])
def test_jit_closest_hit_equals_generic_walk(built, name, tmp_path):
    """The scene-specialised closest-hit kernel (frt_jit_trace: binary32 intervals, the winner's t from its own leaf
    in binary64, the rays it cannot settle handed to the generic walk by k_trace_redo) against k_trace for every
    ray (FRT_JIT_TRACE=0): the canvases are bit-identical (camera rays, reflected rays and, on cornell_gi_16,
    final-gather rays)."""
    ref, _ = _render_env_process(name, {"FRT_JIT_TRACE": "0"}, tmp_path / "g.npy")
    img, _ = _render_env_process(name, {}, tmp_path / "j.npy")
    assert np.array_equal(img, ref), name


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell_direct_64_4x4", "reflect_refract_test_150", "checkered_sphere_dof_100",
                                  "checkered_sphere_jitter_100", "cornell_shipped_48_4x4", "patterns_160x80"])
def test_level0_eyev_from_camera_equals_stored(built, name, tmp_path):
    """Level 0 of a scene without GI does not store its nodes' eye vectors (NodeCols::eye_cam): the shading recomputes
    each one from the node's camera ray (camera_eyev: jitter and thin-lens apertures included). The canvas equals the
    one that stores them (FRT_EYE_CAM=0), bit for bit."""
    ref, _ = _render_env_process(name, {"FRT_EYE_CAM": "0"}, tmp_path / "s.npy")
    img, _ = _render_env_process(name, {}, tmp_path / "c.npy")
    assert np.isfinite(img).all()
    assert np.array_equal(img, ref), name


@pytest.mark.gpu
def test_tile_kernels_on_shipped_multi_row_light(built, tmp_path):
    """The reference's shipped light (cornell_box.yml: 65 535 jittered cache rows, each path node drawing its own row):
    the tile, sub-part and sub-tile stages decide beams against part boxes that hold for every row (CMJ keeps sample
    (u, v) of every row in light cell (u, v)), frt_jit_beam_list against the node's own row. At a fixed seed, row bands
    of the shipped 1920x1080x64 frame through the whole hierarchy, through the node pair kernel alone
    (FRT_JIT_TILE=0) and through the generic walk are bit-identical, and the tile stages ran — with the sub-tile stage's
    list walked ray by ray (the default for multi-row lights), through frt_jit_beam_list (FRT_JIT_NODE_BEAM=1),
    without the sub-tile stage, and with the per-ray kernel's lanes entry-major or node-major (FRT_JIT_NODE_MAJOR)."""
    for rows in ((300, 306), (700, 706)):
        kw = {"row_begin": rows[0], "row_end": rows[1], "seed": 0x5EED}
        ref, st = _render_env_process("cornell_shipped_1920x1080_8x8", {"FRT_JIT": "0"}, tmp_path / "g.npy", **kw)
        assert st[0] == 0
        for i, env in enumerate(({}, {"FRT_JIT_NODE_BEAM": "1"}, {"FRT_JIT_SUBTILE": "0"}, {"FRT_JIT_NODE_MAJOR": "1"},
                                 {"FRT_JIT_NODE_MAJOR": "8"}, {"FRT_JIT_NODE_MAJOR": "64"})):
            img, st = _render_env_process("cornell_shipped_1920x1080_8x8", env, tmp_path / ("t%d.npy" % i), **kw)
            assert st[0] == 1 and st[1] > 0 and st[2] > 0, (env, st)
            assert np.array_equal(img, ref), (rows, env)
        img0, st0 = _render_env_process("cornell_shipped_1920x1080_8x8", {"FRT_JIT_TILE": "0"}, tmp_path / "n.npy", **kw)
        assert st0[0] == 1 and st0[1] == 0, st0
        assert np.array_equal(img0, ref), rows


@pytest.mark.gpu
def test_small_levels_skip_beam_stages_bit_identical(built, tmp_path):
    """Levels with fewer than FRT_JIT_MIN_PAIRS (node, light part) pairs (default 2^18: the deep bounces) walk every
    shadow ray one by one instead of taking the beam stages, whose launches are sized on the host (a round trip
    each). The production default against the stages at every size (FRT_JIT_MIN_PAIRS=0, the test session's
    setting): a band of the headline frame and two small scenes, bit for bit."""
    for name, kw in (("cornell_direct_1920x1080_8x8", {"row_begin": 400, "row_end": 408}),
                     ("reflect_refract_test_150", {}), ("cornell_direct_64_4x4", {})):
        stages, st0 = _render_env_process(name, {"FRT_JIT_MIN_PAIRS": "0"}, tmp_path / "a.npy", **kw)
        default, st1 = _render_env_process(name, {"FRT_JIT_MIN_PAIRS": str(1 << 18)}, tmp_path / "b.npy", **kw)
        assert st0[0] == 1 and st1[0] == 1 and st0[1] > 0
        assert np.array_equal(stages, default), name


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell_direct_64_4x4", "patterns_160x80", "teapot_low_100", "nave_120x150_4x4",
                                  "checkered_torus_120", "reflect_refract_test_150", "bounding_boxes_100x125_4x4",
                                  "area_light_test_100", "checkered_sphere_dof_100", "cornell_gi_24",
                                  "cornell_shipped_48_4x4"])
def test_goldens_under_the_production_default(built, name, tmp_path):
    """The test session walks every level through the beam stages (conftest: FRT_JIT_MIN_PAIRS=0); the shipped default
    (unset: levels under 2^18 (node, part) pairs walk their rays one by one, i.e. every level of these small scenes)
    renders one golden per feature group — CSG cornell, patterns, meshes (OBJ, OBJ+MTL textured, the BVH stand-in),
    torus, refraction, area light, thin-lens aperture, GI, the shipped multi-row light — in a process of its own:
    deterministic goldens within 1e-4 of the reference with its PPM bytes, and every scene bit-identical to the
    session's setting."""
    import hashlib
    from conftest import golden_index, load_golden_canvas
    from fast_ray_tracer_amd.runtime import encode_ppm
    default, st = _render_env_process(name, {"FRT_JIT_MIN_PAIRS": None}, tmp_path / "d.npy")
    stages, _ = _render_env_process(name, {"FRT_JIT_MIN_PAIRS": "0"}, tmp_path / "s.npy")
    assert np.array_equal(default, stages), name
    e = golden_index()[name]
    if not e.get("stochastic"):
        img = default[:, :, :3]
        assert np.abs(img - load_golden_canvas(name)).max() <= 1e-4
        assert hashlib.sha256(encode_ppm(img)).hexdigest() == e["ppm_sha256"]
