#!/bin/bash
# round 6: the node-level specular tail bound (FRT_SHADE_NODE_TAIL): parity over the shading tests (one -k), then
# base vs the nodetail0 variant on the headline and the shipped light
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jit.py tests/test_gpu_parity.py \
    tests/test_gpu_stochastic.py -k "reference_canvas or dense_band or headline or benchmark_scene or row_sorted or lazy_ambient or cornell_gi_24 or cornell_shipped or cfg4 or goldens" \
    > gpurun_out/pytest_r06_o.log 2>&1 || { tail -30 gpurun_out/pytest_r06_o.log; exit 1; }
tail -2 gpurun_out/pytest_r06_o.log
bash tools/gpu_var.sh cornell_direct_1920x1080_8x8 r06_nodetail base nodetail0 base nodetail0 || exit 1
bash tools/gpu_var.sh cornell_shipped_1920x1080_8x8 r06_nodetail_shipped base nodetail0 || exit 1
