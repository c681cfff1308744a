"""render_multi with one, two and four handles on device 0 (FRT_DEVICES "0", "0,0", "0,0,0,0"): the handles render
interleaved rows from host threads of their own, so one handle's host round trips overlap another's kernels. Per
device list: a cold call (upload, level-state allocation) and three warm ones (the kept handles), wall times and
render phases.   python tools/rm_handles_probe.py SCENE   (prints one JSON line)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fast_ray_tracer_amd import build as b  # noqa: E402
from fast_ray_tracer_amd.runtime import Scene, release_render_multi, render_multi, render_multi_phases  # noqa: E402

sc = Scene(os.path.join(b.SCENE_LIB, sys.argv[1] + ".so"), asset_root=os.path.join(ROOT, "tests", "golden", "assets"))
out = {}
ref = None
for devs in ("0", "0,0", "0,0,0,0", "0"):
    release_render_multi()
    runs = []
    for i in range(4):
        t = time.perf_counter()
        img = render_multi(sc, devices=devs)
        runs.append(round(1e3 * (time.perf_counter() - t), 2))
        if ref is None:
            ref = img
        assert (img == ref).all(), devs
    out[devs + ("_again" if devs in out else "")] = {"cold_ms": runs[0], "warm_ms": runs[1:],
                                                     "warm_render_rows_and_copy_ms": render_multi_phases()["render_rows_and_copy"]}
print("JSON" + json.dumps(out))
