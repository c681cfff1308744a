#!/bin/bash
# A/B of device-library builds on the 480x270 GI camera (variants/<name>.so from tools/build_variant.sh; "base" = the
# tree's build): one bench.py process per build, 3 timed frames, the estimate's time per frame.
#   tools/gpu_gi_var.sh <label> base NAME ... [base]
set -o pipefail
mkdir -p gpurun_out
label=$1; shift
out=gpurun_out/gi_ab_${label}.txt
: > $out
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
B="--scene cornell_gi_480x270_8x8 --gi-steps 0 --shipped-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy --steps 3 --warmup 1"
rc=0
for lib in "$@"; do
  if [ "$lib" = base ]; then cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; else cp variants/$lib.so fast_ray_tracer_amd/lib/libfrt_device.so; fi
  timeout -k 10 300 python3 bench.py $B > gpurun_out/gi_ab_${label}.json 2> gpurun_out/gi_ab_${label}.err || { rc=1; tail -5 gpurun_out/gi_ab_${label}.err; break; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
print('%-10s frame %9.2f ms  k_gather_est %9.2f ms  gi %9.2f ms' % (sys.argv[2], d['ms_per_step'], d['sub_ms_per_frame'].get('k_gather_est', 0), d['kernel_ms_per_frame'].get('gi', 0)))
" gpurun_out/gi_ab_${label}.json $lib | tee -a $out
done
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
exit $rc
