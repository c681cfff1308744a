#!/bin/bash
# round 6 evidence: rocprofv3 kernel stats + PMC passes (tools/prof.sh) of the headline, cfg3, cfg4 and shipped
# workloads, summarised per kernel (tools/pmc_summary.py: stamped with the device sources' hash)
#   tools/gpu_r06_prof.sh TAG
set -o pipefail
TAG=${1:-r06}
bash tools/prof.sh ${TAG}_headline cornell_direct_1920x1080_8x8 \
    "k_shade_lit k_prepare frt_jit_sub frt_jit_shadow frt_jit_trace frt_jit_subtile frt_jit_tile k_combine_resolve" || exit 1
bash tools/prof.sh ${TAG}_cfg3 cornell_direct_800_4x4 "k_shade_lit k_prepare frt_jit_sub frt_jit_shadow frt_jit_trace frt_jit_subtile frt_jit_tile" || exit 1
bash tools/prof.sh ${TAG}_cfg4 bounding_boxes_800x1000_4x4 "k_shadow k_trace k_prepare k_shade_lit" || exit 1
bash tools/prof.sh ${TAG}_shipped cornell_shipped_1920x1080_8x8 "frt_jit_shadow k_shade_lit frt_jit_sub k_lit_rows" || exit 1
