#!/bin/bash
# round 4: part / tile sizes on the other cornell workloads (GI with the multi-row light cache, 800x800x16)
set -o pipefail
SC=cornell_gi_480x270_8x8 TESTS="" bash tools/gpu_ab_env.sh pscenes_gi "FRT_JIT=1" "FRT_JIT_PART=1 FRT_JIT_TILE=64" "FRT_JIT_PART=5" && \
SC=cornell_direct_800_4x4 TESTS="" bash tools/gpu_ab_env.sh pscenes_800 "FRT_JIT=1" "FRT_JIT_PART=1 FRT_JIT_TILE=64" "FRT_JIT_PART=3 FRT_JIT_TILE=64"
