#!/bin/bash
# round 4: the scene-specialised closest-hit kernel (frt_jit_trace): bit-identity on the 800x800 frame, the JIT tests,
# the parity tests, then the headline A/B (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/dbg_env_compare.py cornell_direct_800_4x4 "FRT_JIT_TRACE=0" "FRT_JIT_TRACE=1" > gpurun_out/trace_cmp.txt 2>&1
rc=$?
cat gpurun_out/trace_cmp.txt | cut -c1-300
[ $rc -ne 0 ] && exit $rc
TESTS="tests/test_jit.py tests/test_gpu_parity.py" bash tools/gpu_ab_env.sh trace "FRT_JIT_TRACE=0" "FRT_JIT_TRACE=1"
