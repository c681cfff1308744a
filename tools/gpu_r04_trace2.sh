#!/bin/bash
# round 4: frt_jit_trace's undecided share per level, bit-identity, the JIT / parity tests and the headline A/B
# (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
FRT_JIT_TRACE_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-render-multi --gi-steps 0 --scene cornell_direct_1920x1080_8x8 > gpurun_out/trace_stats.log 2>&1 || exit $?
grep "frt_jit_trace level" gpurun_out/trace_stats.log | head -4
timeout -k 10 400 python tools/dbg_env_compare.py cornell_direct_800_4x4 "FRT_JIT_TRACE=0" "FRT_JIT_TRACE=1" > gpurun_out/trace_cmp.txt 2>&1 || exit $?
grep "differ" gpurun_out/trace_cmp.txt
STEPS=3 TESTS="${TESTS-tests/test_jit.py tests/test_gpu_parity.py}" bash tools/gpu_ab_env.sh trace2 "FRT_JIT_TRACE=0" "FRT_JIT_TRACE=1"
