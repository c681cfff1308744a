#!/bin/bash
# round 6 final evidence (a): kernel stats + PMC passes of the headline and cfg3 workloads (tools/prof.sh)
set -o pipefail
bash tools/prof.sh r06_headline cornell_direct_1920x1080_8x8 \
    "k_shade_lit k_prepare frt_jit_sub frt_jit_shadow frt_jit_trace frt_jit_subtile frt_jit_tile k_combine_resolve" || exit 1
bash tools/prof.sh r06_cfg3 cornell_direct_800_4x4 "k_shade_lit k_prepare frt_jit_sub frt_jit_shadow frt_jit_trace frt_jit_subtile frt_jit_tile" || exit 1
