"""One rank's rows (r, r+N, ...) of the headline frame on one handle, against two handles on the same GPU rendering
alternate rows of that set concurrently from two host threads (each handle its own stream: one's host round trips
overlap the other's kernels). Best of K frames each.   python tools/dual_probe.py [K]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fast_ray_tracer_amd import build  # noqa: E402
from fast_ray_tracer_amd.runtime import GpuRenderer, Scene  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
sc = Scene(os.path.join(build.SCENE_LIB, "cornell_direct_1920x1080_8x8.so"),
           asset_root=os.path.join(ROOT, "tests", "golden", "assets"))
H, W = sc.height, sc.width
a, b = GpuRenderer(sc, device=0), GpuRenderer(sc, device=0)
for N in (1, 2, 4, 8):
    rows = (H + N - 1) // N
    one = torch.zeros((rows, W, 4), dtype=torch.float64, device="cuda")
    ha = torch.zeros(((rows + 1) // 2, W, 4), dtype=torch.float64, device="cuda")
    hb = torch.zeros(((rows + 1) // 2, W, 4), dtype=torch.float64, device="cuda")
    best1 = best2 = 1e9
    for i in range(K + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.render_into(one.data_ptr(), row_begin=0, row_end=H, row_stride=N, batch_samples=1 << 27)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ta = threading.Thread(target=a.render_into, args=(ha.data_ptr(),),
                              kwargs=dict(row_begin=0, row_end=H, row_stride=2 * N, batch_samples=1 << 27))
        tb = threading.Thread(target=b.render_into, args=(hb.data_ptr(),),
                              kwargs=dict(row_begin=N, row_end=H, row_stride=2 * N, batch_samples=1 << 27))
        ta.start()
        tb.start()
        ta.join()
        tb.join()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if i > 0:
            best1 = min(best1, t1 - t0)
            best2 = min(best2, t2 - t1)
    na = (rows + 1) // 2
    same = torch.equal(one[0::2], ha[:na]) and torch.equal(one[1::2], hb[:rows - na])
    print("N=%d: one handle %.3f ms, two handles %.3f ms, rows equal: %s" % (N, 1e3 * best1, 1e3 * best2, same), flush=True)
