#!/bin/bash
# round 4: the sub-tile pass (frt_jit_subtile between frt_jit_sub and frt_jit_beam_list): bit-identity on the 800x800
# frame, the JIT tests, then sub-tile / tile sizes on the headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/dbg_env_compare.py cornell_direct_800_4x4 "FRT_JIT=0" "FRT_JIT=1" "FRT_JIT_SUBTILE=4 FRT_JIT_TILE=32" "FRT_JIT_SUBTILE=32" > gpurun_out/subtile_cmp.txt 2>&1 && \
TESTS="tests/test_jit.py" bash tools/gpu_ab_env.sh subtile "FRT_JIT_SUBTILE=0" "FRT_JIT=1" "FRT_JIT_SUBTILE=4" "FRT_JIT_SUBTILE=16" "FRT_JIT_SUBTILE=32" "FRT_JIT_TILE=32 FRT_JIT_SUBTILE=8" "FRT_JIT_TILE=32 FRT_JIT_SUBTILE=4" "FRT_JIT=1"
