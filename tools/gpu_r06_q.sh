#!/bin/bash
# round 6: kernel trace of the headline after the parent-order sort; A/B of the sort's key width (FRT_QUEUE_SORT_SHIFT)
set -o pipefail
mkdir -p gpurun_out
bash tools/kt.sh r06q_headline cornell_direct_1920x1080_8x8 || exit 1
bash tools/gpu_ab.sh cornell_direct_1920x1080_8x8 r06_sort_shift "FRT_QUEUE_SORT_SHIFT=0" "FRT_QUEUE_SORT_SHIFT=6" \
    "FRT_QUEUE_SORT_SHIFT=0" "FRT_QUEUE_SORT_SHIFT=6" || exit 1
bash tools/gpu_ab.sh cornell_shipped_1920x1080_8x8 r06_sort_shift_shipped "FRT_QUEUE_SORT_SHIFT=0" "FRT_QUEUE_SORT_SHIFT=6" || exit 1
