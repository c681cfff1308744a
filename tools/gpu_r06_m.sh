#!/bin/bash
# round 6: the secondary levels' queues in parent order (FRT_QUEUE_SORT) and the ballot-gated closest-hit deferral:
# parity (one -k over the files), then headline / shipped / cfg4 A/B of the queue order
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jit.py tests/test_gpu_parity.py \
    tests/test_gpu_stochastic.py -k "closest_hit or equals_generic or reference_canvas or headline or benchmark_scene or lazy_ambient or gather or cornell_gi_24 or cornell_shipped or cfg4 or mesh_search or split or glass" \
    > gpurun_out/pytest_r06_m.log 2>&1 || { tail -30 gpurun_out/pytest_r06_m.log; exit 1; }
tail -2 gpurun_out/pytest_r06_m.log
bash tools/gpu_ab.sh cornell_direct_1920x1080_8x8 r06_queue_sort "FRT_QUEUE_SORT=0" "FRT_QUEUE_SORT=1" "FRT_QUEUE_SORT=0" \
    "FRT_QUEUE_SORT=1" || exit 1
bash tools/gpu_ab.sh cornell_shipped_1920x1080_8x8 r06_queue_sort_shipped "FRT_QUEUE_SORT=0" "FRT_QUEUE_SORT=1" || exit 1
bash tools/gpu_ab.sh bounding_boxes_800x1000_4x4 r06_queue_sort_cfg4 "FRT_QUEUE_SORT=0" "FRT_QUEUE_SORT=1" || exit 1
