#!/bin/bash
# round 6, first pass: the new paths' GPU tests (staged row-ordered shading, node-major per-ray lanes, render_multi
# keys / release / lock, goldens under the production default), then shipped-frame A/B of the two switches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "row_sorted or keeps_handles or concurrent or failure" \
    tests/test_jit.py -k "shipped or tile_and_sub or production_default" \
    tests/test_gpu_stochastic.py -k "shipped" > gpurun_out/pytest_r06_a.log 2>&1 || { tail -30 gpurun_out/pytest_r06_a.log; exit 1; }
tail -3 gpurun_out/pytest_r06_a.log
bash tools/gpu_ab.sh cornell_shipped_1920x1080_8x8 r06_shipped "FRT_SHADE_STAGE=0" "FRT_SHADE_STAGE=1" \
    "FRT_JIT_NODE_MAJOR=4" "FRT_JIT_NODE_MAJOR=16" "FRT_JIT_NODE_MAJOR=64" "FRT_SHADE_STAGE=0"
