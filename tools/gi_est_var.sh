#!/bin/bash
# round 5: k_gather_est per device-library build on the GI 480x270 frame (variants/<name>.so; "base" = the tree's
# build): tools/gi_est_var.sh base NAME ...   (one process per build: a warm frame, then a timed one)
set -o pipefail
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
for lib in "$@"; do
  if [ "$lib" = base ]; then cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; else cp variants/$lib.so fast_ray_tracer_amd/lib/libfrt_device.so; fi
  timeout -k 10 300 python -c "
import sys, time
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from conftest import load_scene
from fast_ray_tracer_amd.runtime import GpuRenderer
r = GpuRenderer(load_scene('${SC:-cornell_gi_480x270_8x8}'))
for i in range(2):
    t0 = time.perf_counter(); img, st = r.render(seed=0x61000 + i, stats=True); t = 1e3 * (time.perf_counter() - t0)
d = st.as_dict()
print('$lib: frame %.0f ms, k_gather_est %.1f ms (%d launches), gather rays %d' % (t, d['sub_ms'].get('k_gather_est', 0), d['sub_launches'].get('k_gather_est', 0), d['gather_rays']))
" || { cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; exit 1; }
done
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
