#!/bin/bash
# round 6: k_shade_lit occupancy (FRT_SHADE_WAVES 3 / 5 builds against the tree's 4) on the headline and shipped
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_var.sh cornell_direct_1920x1080_8x8 r06_shw base shw3 shw5 base || exit 1
bash tools/gpu_var.sh cornell_shipped_1920x1080_8x8 r06_shw_shipped base shw3 shw5 || exit 1
