#!/bin/bash
# round 6 (late): k_shade_lit occupancy x point pairing on the tree with the one-reciprocal BRDF: 3 waves per SIMD
# (variants/w3.so), two points per step at 4 (pair4) and 3 (pair3) waves, headline frame (tools/gpu_var.sh)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_var.sh cornell_direct_1920x1080_8x8 shade_occ base w3 pair4 pair3 base || exit 1
cat gpurun_out/ab_shade_occ_all.txt
