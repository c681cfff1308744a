#!/bin/bash
# round 4: part size around 8 with tile sizes and occupancy, headline A/B
set -o pipefail
TESTS="" bash tools/gpu_ab_env.sh parts2 "FRT_JIT_PART=8" "FRT_JIT_PART=4" "FRT_JIT_PART=5" "FRT_JIT_PART=6" "FRT_JIT_PART=8 FRT_JIT_TILE=64" "FRT_JIT_PART=8 FRT_JIT_TILE=16" "FRT_JIT_PART=8 FRT_JIT_WAVES=8" "FRT_JIT_PART=7 FRT_JIT_TILE=64" "FRT_JIT_PART=8 FRT_JIT_ORDER=2" "FRT_JIT_PART=8"
