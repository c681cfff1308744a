#!/bin/bash
# round 6 final evidence (b): kernel stats + PMC passes of cfg4 and the shipped light (tools/prof.sh)
set -o pipefail
bash tools/prof.sh r06_cfg4 bounding_boxes_800x1000_4x4 "k_shadow k_trace k_prepare k_shade_lit" || exit 1
bash tools/prof.sh r06_shipped cornell_shipped_1920x1080_8x8 "frt_jit_shadow k_shade_lit frt_jit_sub k_lit_rows" || exit 1
