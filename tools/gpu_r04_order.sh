#!/bin/bash
# round 4: same-axis slab order in the pair kernels (FRT_JIT_ORDER 0/1/2): bit-identity on the 800x800 frame, the
# JIT / parity tests, then the headline A/B (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/dbg_env_compare.py cornell_direct_800_4x4 "FRT_JIT=0" "FRT_JIT_ORDER=0" "FRT_JIT_ORDER=1" "FRT_JIT_ORDER=2" > gpurun_out/order_cmp.txt 2>&1 && \
TESTS="${TESTS-tests/test_jit.py tests/test_gpu_parity.py}" bash tools/gpu_ab_env.sh order "FRT_JIT_ORDER=0" "FRT_JIT_ORDER=1" "FRT_JIT_ORDER=2" "FRT_JIT_ORDER=0" "FRT_JIT_ORDER=1" "FRT_JIT_ORDER=2"
