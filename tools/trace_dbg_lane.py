"""Print the scene-specialised closest hit's walk of one camera ray (FRT_JIT_TRACE_DBG): the nodes where it becomes
undecidable.   python tools/trace_dbg_lane.py SCENE X Y [SUB]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_scene  # noqa: E402

sc = load_scene(sys.argv[1])
x, y = int(sys.argv[2]), int(sys.argv[3])
sub = int(sys.argv[4]) if len(sys.argv) > 4 else 0
os.environ["FRT_JIT_TRACE_DBG"] = str(x * sc.spp + sub)  # (the kernel's index within the batch: row y alone)
os.environ["FRT_JIT_CACHE"] = "0"
from fast_ray_tracer_amd.runtime import GpuRenderer  # noqa: E402

r = GpuRenderer(sc)
r.render(row_begin=y, row_end=y + 1)
