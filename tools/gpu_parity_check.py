"""Quick GPU-vs-golden parity sweep (developer tool; the real tests live in tests/)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from fast_ray_tracer_amd import build
from fast_ray_tracer_amd.runtime import Scene, GpuRenderer

G = os.path.join(ROOT, "tests", "golden")
idx = json.load(open(os.path.join(G, "golden.json")))
for name, e in sorted(idx.items()):
    if "canvas" not in e:
        continue
    sc = Scene(build.build_scene(os.path.join(G, "scenes", name + ".c")), asset_root=os.path.join(G, "assets"))
    try:
        r = GpuRenderer(sc)
    except RuntimeError as ex:
        print(f"{name:28s} SKIP {ex}", flush=True)
        continue
    t = time.time()
    img, st = r.render(stats=True)
    dt = time.time() - t
    ref = np.load(os.path.join(G, e["canvas"]))["canvas"]
    d = np.abs(img[:, :, :3] - ref)
    print(f"{name:28s} max|d|={d.max():.3e} n>1e-4={int((d>1e-4).sum())} mismatches={int((d>0).sum())} "
          f"bitexact={np.array_equal(img[:, :, :3], ref)} {dt*1e3:.1f}ms {st.as_dict()['kernel_ms']}", flush=True)
    r.close()
