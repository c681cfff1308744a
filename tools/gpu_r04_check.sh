#!/bin/bash
# round 4: bit-identity of the JIT path on the 800x800 frame against the generic walk, the JIT / parity tests, then
# the headline timing (run via gpurun from the repo root): TAG=name bash tools/gpu_r04_check.sh [env settings...]
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-check}
timeout -k 10 400 python tools/dbg_env_compare.py cornell_direct_800_4x4 "FRT_JIT=0" "FRT_JIT=1" > gpurun_out/${TAG}_cmp.txt 2>&1 && \
TESTS="${TESTS-tests/test_jit.py tests/test_gpu_parity.py}" bash tools/gpu_ab_env.sh $TAG "FRT_JIT=1" "$@"
