#!/usr/bin/env python3
"""render_multi of the headline frame with several handles on one GPU (FRT_DEVICES=0,0,...: each handle its own host
thread and stream, rows interleaved) against one handle: whether the shadow pass's host round trips leave the GPU idle
(run via gpurun from the repo root):  python tools/rm_streams.py 0 0,0 0,0,0"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_scene  # noqa: E402
from fast_ray_tracer_amd.runtime import render_multi  # noqa: E402

sc = load_scene(os.environ.get("SC", "cornell_direct_1920x1080_8x8"))
ref = None
for devs in sys.argv[1:]:
    render_multi(sc, devices=devs)  # warm: upload, JIT module, first allocations
    ts = []
    for _ in range(int(os.environ.get("REPS", "3"))):
        t0 = time.perf_counter()
        img = render_multi(sc, devices=devs)
        ts.append(1e3 * (time.perf_counter() - t0))
    same = "" if ref is None else ("identical" if (img == ref).all() else "DIFFERENT")
    ref = img if ref is None else ref
    print("devices %-8s ms per frame (wall, upload included) %s %s" % (devs, " ".join("%.1f" % t for t in ts), same), flush=True)
