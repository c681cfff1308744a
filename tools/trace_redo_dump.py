"""Where the scene-specialised closest hit hands camera rays to the generic walk: renders the headline camera with
FRT_JIT_TRACE_STATS / FRT_JIT_TRACE_DUMP and histograms the undecided level-0 rays by pixel region and sub-sample.
   python tools/trace_redo_dump.py SCENE OUT.npy"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["FRT_JIT_TRACE_STATS"] = "1"
os.environ["FRT_JIT_TRACE_DUMP"] = "/tmp/frt_trace_redo.bin"
from conftest import load_scene  # noqa: E402
from fast_ray_tracer_amd.runtime import GpuRenderer  # noqa: E402

sc = load_scene(sys.argv[1])
r = GpuRenderer(sc)
r.render(batch_samples=1 << 27)
idx = np.fromfile("/tmp/frt_trace_redo.bin", dtype=np.int32).astype(np.int64)
spp = sc.spp
pix = idx // spp
sub = idx % spp
y, x = pix // sc.width, pix % sc.width
np.save(sys.argv[2], np.stack([x, y, sub]).astype(np.int32))
print("undecided", len(idx), "of", sc.width * sc.height * spp)
H, _, _ = np.histogram2d(y, x, bins=[12, 16], range=[[0, sc.height], [0, sc.width]])
np.set_printoptions(linewidth=200)
print((H / (sc.height / 12 * sc.width / 16 * spp) * 100).round(1))
print("by sub-sample", np.bincount(sub, minlength=spp)[:16])
