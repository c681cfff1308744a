#!/bin/bash
# round 6: dense spawn (FRT_QUEUE_SORT=2): queue-order parity + the shading / golden tests (one -k), then A/B of
# the queue modes 1 (radix sort) and 2 (dense) on the headline, shipped and cfg4, and a kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jit.py tests/test_gpu_parity.py \
    tests/test_gpu_stochastic.py -k "queue_order or reference_canvas or dense_band or headline or benchmark_scene or lazy_ambient or cornell_gi_24 or cornell_shipped or cfg4 or gather" \
    > gpurun_out/pytest_r06_r.log 2>&1 || { tail -30 gpurun_out/pytest_r06_r.log; exit 1; }
tail -2 gpurun_out/pytest_r06_r.log
bash tools/gpu_ab.sh cornell_direct_1920x1080_8x8 r06_dense "FRT_QUEUE_SORT=1" "FRT_QUEUE_SORT=2" "FRT_QUEUE_SORT=1" \
    "FRT_QUEUE_SORT=2" || exit 1
bash tools/gpu_ab.sh cornell_shipped_1920x1080_8x8 r06_dense_shipped "FRT_QUEUE_SORT=1" "FRT_QUEUE_SORT=2" || exit 1
bash tools/gpu_ab.sh bounding_boxes_800x1000_4x4 r06_dense_cfg4 "FRT_QUEUE_SORT=1" "FRT_QUEUE_SORT=2" || exit 1
bash tools/kt.sh r06r_headline cornell_direct_1920x1080_8x8 || exit 1
