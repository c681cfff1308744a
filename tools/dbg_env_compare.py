#!/usr/bin/env python3
"""Render one golden scene on the GPU under several environment settings (one process each) and compare the
canvases with the first setting's, bit for bit (debug aid for engine switches that must not change a pixel).

  python tools/dbg_env_compare.py SCENE "FRT_JIT=0" "FRT_JIT_TILE=0" "FRT_JIT_TILE=8" ...
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name = sys.argv[1]
outs = []
for i, e in enumerate(sys.argv[2:]):
    env = dict(os.environ)
    for kv in e.split():
        k, v = kv.split("=", 1)
        env[k] = v
    path = "/tmp/frt_dbg_%d.npy" % i
    code = ("import sys, numpy as np; sys.path.insert(0, %r); from fast_ray_tracer_amd import build as b; "
            "from fast_ray_tracer_amd.runtime import Scene, GpuRenderer; "
            "sc = Scene(b.build_scene(%r), asset_root=%r); img, st = GpuRenderer(sc).render(stats=True); "
            "np.save(%r, img); d = st.as_dict(); print({k: d[k] for k in ('shadow_jit', 'shadow_rays_walked', "
            "'shadow_tile_pairs', 'shadow_tile_mixed', 'shadow_pairs', 'shadow_pairs_mixed', 'errors')})"
            % (ROOT, os.path.join(ROOT, "tests/golden/scenes", name + ".c"), os.path.join(ROOT, "tests/golden/assets"), path))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(e, "rc", p.returncode, p.stdout.strip().splitlines()[-1:] if p.stdout else "", p.stderr[-400:] if p.returncode else "")
    if p.returncode:
        sys.exit(1)
    outs.append(np.load(path))
    if i:
        d = np.abs(outs[i] - outs[0])
        bad = np.argwhere(d.max(axis=2) > 0)
        print("  vs first: %d pixels differ, max %.3g; first: %s" % (len(bad), d.max(), bad[:8].tolist()))
