#!/bin/bash
# round 6 (late): the final gather's hemisphere rays through frt_jit_trace (FRT_GATHER_JIT=1) against the generic walk,
# cornell_gi_480x270_8x8 (3 frames per process), then one full-size GI frame each; the GI GPU tests with the knob on
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/gi_jit.txt
for v in FRT_NOP=0 FRT_GATHER_JIT=1 FRT_NOP=0 FRT_GATHER_JIT=1; do
  env $v timeout -k 10 300 python3 bench.py --scene cornell_gi_480x270_8x8 --gi-steps 0 --shipped-steps 0 --no-cpu-baseline \
      --no-render-multi --no-scaling-proxy --steps 3 --warmup 1 > gpurun_out/gi_jit.json 2> gpurun_out/gi_jit.err || { tail -5 gpurun_out/gi_jit.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
print('%-18s 480x270 frame %9.2f ms  k_gather_est %9.2f ms  gi %9.2f ms  sub %s' % (sys.argv[2], d['ms_per_step'], d['sub_ms_per_frame'].get('k_gather_est', 0), d['kernel_ms_per_frame'].get('gi', 0), {k: v for k, v in d['sub_ms_per_frame'].items() if 'gather' in k or 'trace' in k}))
" gpurun_out/gi_jit.json $v | tee -a gpurun_out/gi_jit.txt
done
FRT_GATHER_JIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_stochastic.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "gi or gather" > gpurun_out/pytest_gatherjit.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gatherjit.log; exit $rc
