import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
ORACLE_DIR = os.path.join(ROOT, "oracle")
if ORACLE_DIR not in sys.path:
    sys.path.insert(0, ORACLE_DIR)

# The test scenes are small: every level of them would skip the shadow pass's beam stages (frt_engine.hip
# launch_shadow: levels under FRT_JIT_MIN_PAIRS (node, light part) pairs walk their rays one by one). The tests
# exercise the stages at every size; test_jit.py::test_small_levels_skip_beam_stages_bit_identical and
# test_goldens_under_the_production_default (one golden per feature group, in processes without this override) check
# the shipped default.
os.environ.setdefault("FRT_JIT_MIN_PAIRS", "0")

GOLDEN = os.path.join(ROOT, "tests", "golden")
ASSETS = os.path.join(GOLDEN, "assets")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")


def golden_index():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def canvas_goldens():
    return sorted(n for n, e in golden_index().items() if "canvas" in e)


@pytest.fixture(scope="session")
def built():
    from fast_ray_tracer_amd import build
    build.build_host()
    build.build_oracle()
    return build


_scenes = {}


def load_scene(name):
    """Capture a golden scene (built once per session)."""
    if name not in _scenes:
        from fast_ray_tracer_amd import build
        from fast_ray_tracer_amd.runtime import Scene
        so = build.build_scene(os.path.join(GOLDEN, "scenes", name + ".c"))
        _scenes[name] = Scene(so, asset_root=ASSETS)
    return _scenes[name]


def fresh_scene(name):
    """Capture a golden scene anew (not cached): the libc RNG state right after its main()."""
    from fast_ray_tracer_amd import build
    from fast_ray_tracer_amd.runtime import Scene
    return Scene(build.build_scene(os.path.join(GOLDEN, "scenes", name + ".c")), asset_root=ASSETS)


def load_golden_canvas(name):
    import numpy as np
    e = golden_index()[name]
    return np.load(os.path.join(GOLDEN, e["canvas"]))["canvas"]
