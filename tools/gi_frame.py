"""One GI frame (a warm one first when --warm): the program rocprofv3 runs in tools/pmc_gi_sort.sh.
python tools/gi_frame.py SCENE [--warm]"""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
from conftest import load_scene  # noqa: E402
from fast_ray_tracer_amd.runtime import GpuRenderer  # noqa: E402

r = GpuRenderer(load_scene(sys.argv[1]))
for i in range(2 if "--warm" in sys.argv else 1):
    t0 = time.perf_counter()
    img, st = r.render(seed=0x61000 + i, stats=True)
    t = 1e3 * (time.perf_counter() - t0)
d = st.as_dict()
print("frame %.0f ms, k_gather_est %.1f ms, gather rays %d" % (t, d["sub_ms"].get("k_gather_est", 0), d["gather_rays"]))
