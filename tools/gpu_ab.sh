#!/bin/bash
# headline-style A/B of engine knobs on one scene: tools/gpu_ab.sh <scene> <label> "<ENV=..>" ["<ENV=..>" ...]
# (each variant one bench.py process, steps 5, the stats frame's kernel split; a line per variant in gpurun_out/ab_<label>.txt)
set -o pipefail
mkdir -p gpurun_out
sc=$1; label=$2; shift 2
out=gpurun_out/ab_${label}.txt
: > $out
for v in "$@"; do
  env $v timeout -k 10 300 python -u bench.py --scene $sc --steps 5 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi \
    --no-scaling-proxy --shipped-steps 0 > gpurun_out/ab_${label}.json 2> gpurun_out/ab_${label}.err || { tail -20 gpurun_out/ab_${label}.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); sp=d['shadow_pass']
sub = d['sub_ms_per_frame']
print('%-40s ms %8.3f shadow %7.3f shade %6.3f (lit %6.3f sort %5.3f) prepare %6.3f | %s | node_pairs %s walked %s lit %s' % (sys.argv[2], d['ms_per_step'], d['kernel_ms_per_frame']['shadow'], d['kernel_ms_per_frame']['shade'], sub.get('k_shade_lit', 0), sub.get('k_lit_sort', 0), d['kernel_ms_per_frame']['prepare'], ' '.join('%s %.2f' % (k[8:], v) for k, v in sp['kernels_ms_per_frame'].items()), sp['node_pairs'], sp['shadow_rays_walked_per_ray'], d.get('lit_nodes_per_frame')))
" gpurun_out/ab_${label}.json "$v" | tee -a $out
done
