#!/bin/bash
# round 4: rays per lane of the per-ray kernel (FRT_JIT_REP): bit-identity on the 800x800 frame, then the headline A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/dbg_env_compare.py cornell_direct_800_4x4 "FRT_JIT=0" "FRT_JIT_REP=2" "FRT_JIT_REP=4" "FRT_JIT_REP=8 FRT_JIT_WAVES=7" > gpurun_out/rep_cmp.txt 2>&1 && \
TESTS="" bash tools/gpu_ab_env.sh rep "FRT_JIT_REP=1" "FRT_JIT_REP=2" "FRT_JIT_REP=4" "FRT_JIT_REP=2 FRT_JIT_WAVES=7" "FRT_JIT_REP=4 FRT_JIT_WAVES=7" "FRT_JIT_REP=8 FRT_JIT_WAVES=7" "FRT_JIT_REP=4 FRT_JIT_WAVES=6"
