#!/bin/bash
# round 5: the GI frame with the gather requests in gather order (FRT_GATHER_SORT=0) and sorted (default), one
# process each (a warm frame, then a timed one): SC=<scene> tools/gi_sort_ab.sh
set -o pipefail
for mode in 0 -1 0 -1; do
  FRT_GATHER_SORT=$mode timeout -k 10 ${TMO:-300} python -c "
import sys, time
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from conftest import load_scene
from fast_ray_tracer_amd.runtime import GpuRenderer
r = GpuRenderer(load_scene('${SC:-cornell_gi_480x270_8x8}'))
for i in range(2):
    t0 = time.perf_counter(); img, st = r.render(seed=0x61000 + i, stats=True); t = 1e3 * (time.perf_counter() - t0)
d = st.as_dict()
print('FRT_GATHER_SORT=$mode: frame %.0f ms, k_gather_est %.1f ms (%d launches), gather rays %d' % (t, d['sub_ms'].get('k_gather_est', 0), d['sub_launches'].get('k_gather_est', 0), d['gather_rays']))
" || exit 1
done
