"""The drop-in's per-process cost, measured in a fresh process (round 5): the HIP runtime's own initialisation
(hipSetDevice + hipFree(0) + a 1 MB hipMalloc, through libamdhip64 alone), loading libfrt_device / libfrt_host, the
scene build (main() in capture mode), then render_multi with its phases (frt_render_multi_phases).

  python tools/rm_probe.py SCENE [--init-first]     (prints one JSON line)"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
out = {}
t0 = time.perf_counter()
if "--init-first" in sys.argv:
    hip = ctypes.CDLL("libamdhip64.so")
    t = time.perf_counter()
    hip.hipSetDevice(0)
    out["hip_set_device_ms"] = 1e3 * (time.perf_counter() - t)
    t = time.perf_counter()
    hip.hipFree(ctypes.c_void_p(0))
    out["hip_free0_ms"] = 1e3 * (time.perf_counter() - t)
    p = ctypes.c_void_p()
    t = time.perf_counter()
    hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20))
    out["hip_malloc_1mb_ms"] = 1e3 * (time.perf_counter() - t)
    hip.hipFree(p)
t = time.perf_counter()
from fast_ray_tracer_amd import build as b  # noqa: E402
from fast_ray_tracer_amd.runtime import Scene, jit_cache_stats, render_multi, render_multi_phases  # noqa: E402
out["import_ms"] = 1e3 * (time.perf_counter() - t)
name = sys.argv[1]
t = time.perf_counter()
sc = Scene(os.path.join(b.SCENE_LIB, name + ".so"), asset_root=os.path.join(ROOT, "tests", "golden", "assets"))
out["scene_main_ms"] = 1e3 * (time.perf_counter() - t)
t = time.perf_counter()
render_multi(sc, devices="0")
out["render_multi_ms"] = 1e3 * (time.perf_counter() - t)
out["phases"] = render_multi_phases()
out["compiles"] = jit_cache_stats()["compiles"]
t = time.perf_counter()
render_multi(sc, devices="0")
out["render_multi_warm_ms"] = 1e3 * (time.perf_counter() - t)
out["phases_warm"] = render_multi_phases()
out["process_ms"] = 1e3 * (time.perf_counter() - t0)
print("JSON" + json.dumps(out))
