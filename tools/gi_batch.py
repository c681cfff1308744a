#!/usr/bin/env python3
"""GI frames of the GI workload at several samples per batch, one process each: a warm frame, then a timed one (fresh
photon maps in each, as bench.py times them) (run via gpurun from the repo root):  python tools/gi_batch.py 8388608 ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, time
sys.path.insert(0, %r); sys.path.insert(0, %r)
from conftest import load_scene
from fast_ray_tracer_amd.runtime import GpuRenderer
sc = load_scene(%r)
r = GpuRenderer(sc)
b = int(sys.argv[1])
ts = []
for i in range(2):
    t0 = time.perf_counter(); img, st = r.render(seed=0x61000 + i, batch_samples=b, stats=True); ts.append(1e3 * (time.perf_counter() - t0))
    d = st.as_dict()
print("frames ms %%s | gi kernel ms %%.0f" %% (" ".join("%%.0f" %% t for t in ts), d["kernel_ms"].get("gi", 0.0)))
""" % (ROOT, os.path.join(ROOT, "tests"), os.environ.get("SC", "cornell_gi_1920x1080_8x8"))
for b in sys.argv[1:]:
    p = subprocess.run([sys.executable, "-c", CODE, b], capture_output=True, text=True, timeout=900)
    print("batch %10s:" % b, (p.stdout.strip().splitlines() or [""])[-1], p.stderr[-300:] if p.returncode else "", flush=True)
