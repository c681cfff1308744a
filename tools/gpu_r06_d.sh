#!/bin/bash
# round 6, fourth pass: paired light points in the shading (FRT_SHADE_PAIR) — parity (goldens, the headline rows and
# dense band, the math sequences, lazy ambient, row-sorted shading), then the headline and shipped frames per build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "reference_canvas or headline or benchmark_scene or math_core or lazy_ambient or row_sorted" \
    > gpurun_out/pytest_r06_d.log 2>&1 || { tail -30 gpurun_out/pytest_r06_d.log; exit 1; }
tail -2 gpurun_out/pytest_r06_d.log
bash tools/gpu_var.sh cornell_direct_1920x1080_8x8 r06_pair base nopair pairw3 base nopair || exit 1
bash tools/gpu_var.sh cornell_shipped_1920x1080_8x8 r06_pair_shipped base nopair
