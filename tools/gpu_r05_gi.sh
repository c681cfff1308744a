#!/bin/bash
# round 5: GI frame A/B (cornell_gi_1920x1080_8x8 as bench.py times it): tools/gpu_r05_gi.sh <label> "<ENV=..>" ...
set -o pipefail
mkdir -p gpurun_out
label=$1; shift
out=gpurun_out/gi_${label}.txt
: > $out
for v in "$@"; do
  env $v timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --gi-steps 1 --shipped-steps 0 --no-cpu-baseline \
    --no-render-multi --no-scaling-proxy > gpurun_out/gi_${label}.json 2> gpurun_out/gi_${label}.err || { tail -20 gpurun_out/gi_${label}.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().splitlines()[-1])['gi']
print('%-40s GI ms %9.1f gather_est %9.1f (%d launches) shadow %.1f shade %.1f photon %.1f' % (sys.argv[2], d['ms_per_step'], d['gather_est']['ms_per_frame'], d['gather_est']['launches'], d['kernel_ms_per_frame']['shadow'], d['kernel_ms_per_frame']['shade'], d['photon_ms']))
" gpurun_out/gi_${label}.json "$v" | tee -a $out
done
