#!/bin/bash
# round 4: part size (samples per light part) and tile size sweep on the round-4 build, headline A/B
set -o pipefail
TESTS="" bash tools/gpu_ab_env.sh parts "FRT_JIT_PART=13" "FRT_JIT_PART=7" "FRT_JIT_PART=8" "FRT_JIT_PART=9" "FRT_JIT_PART=10" "FRT_JIT_PART=11" "FRT_JIT_PART=12" "FRT_JIT_PART=14" "FRT_JIT_PART=15" "FRT_JIT_PART=10 FRT_JIT_TILE=64" "FRT_JIT_PART=10 FRT_JIT_TILE=16"
