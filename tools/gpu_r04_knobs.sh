#!/bin/bash
# round 4: the JIT knobs again on the round-4 build (occupancy, decision representation, part size), headline A/B
set -o pipefail
TESTS="" bash tools/gpu_ab_env.sh knobs "FRT_JIT=1" "FRT_JIT_WAVES=8" "FRT_JIT_BEAM_WAVES=8" "FRT_JIT_U32=2" "FRT_JIT_U32=0" "FRT_JIT_PART=13" "FRT_JIT_PART=20" "FRT_JIT_PART=25" "FRT_JIT=1"
