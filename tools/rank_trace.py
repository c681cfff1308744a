"""One rank's share of an N-rank frame (rows r, r+N, ...) rendered repeatedly on one GPU, for a kernel trace of its
fixed per-frame costs (round 5: the scaling proxy's N = 8 rank).   python tools/rank_trace.py [N] [frames]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fast_ray_tracer_amd import build  # noqa: E402
from fast_ray_tracer_amd.runtime import GpuRenderer, Scene  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 6
sc = Scene(os.path.join(build.SCENE_LIB, "cornell_direct_1920x1080_8x8.so"),
           asset_root=os.path.join(ROOT, "tests", "golden", "assets"))
r = GpuRenderer(sc, device=0)
out = torch.zeros(((sc.height + n - 1) // n, sc.width, 4), dtype=torch.float64, device="cuda")
for i in range(frames):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.render_into(out.data_ptr(), row_begin=0, row_end=sc.height, row_stride=n, batch_samples=1 << 27)
    torch.cuda.synchronize()
    print("frame %d: %.3f ms" % (i, 1e3 * (time.perf_counter() - t0)), flush=True)
