#!/bin/bash
# round 6, third pass: GI estimate builds; the node-major lanes on the single-row headline; the shipped defaults
set -o pipefail
bash tools/gpu_gi_var.sh r06_est base scan2 scan4 sqrt1 w3 base || exit 1
bash tools/gpu_ab.sh cornell_direct_1920x1080_8x8 r06_headline_nm "FRT_JIT_NODE_MAJOR=1" "FRT_JIT_NODE_MAJOR=4" "FRT_JIT_NODE_MAJOR=2" "FRT_JIT_NODE_MAJOR=1" || exit 1
bash tools/gpu_ab.sh cornell_shipped_1920x1080_8x8 r06_shipped_defaults "FRT_X=0"
