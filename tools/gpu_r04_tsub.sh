#!/bin/bash
# round 4: the sub-part pass at the tile level (frt_jit_sub between frt_jit_tile and frt_jit_beam_list): bit-identity on
# the 800x800 frame, the JIT tests, then part / sub-part / tile sizes on the headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/dbg_env_compare.py cornell_direct_800_4x4 "FRT_JIT=0" "FRT_JIT_SUB=16 FRT_JIT_PART=16 FRT_JIT_TILE=64" "FRT_JIT_SUB=4" "FRT_JIT_SUB=8 FRT_JIT_PART=16 FRT_JIT_TILE=64" > gpurun_out/tsub_cmp.txt 2>&1 && \
TESTS="tests/test_jit.py" bash tools/gpu_ab_env.sh tsub "FRT_JIT_PART=1 FRT_JIT_TILE=64" "FRT_JIT_PART=16 FRT_JIT_SUB=16 FRT_JIT_TILE=64" "FRT_JIT_PART=8 FRT_JIT_SUB=8 FRT_JIT_TILE=64" "FRT_JIT_PART=32 FRT_JIT_SUB=32 FRT_JIT_TILE=64" "FRT_JIT_PART=16 FRT_JIT_SUB=8 FRT_JIT_TILE=64" "FRT_JIT_PART=12 FRT_JIT_SUB=4 FRT_JIT_TILE=64" "FRT_JIT_PART=16 FRT_JIT_SUB=16 FRT_JIT_TILE=32"
