#!/bin/bash
# round 6: the specular tail test from binary32 n.h (FRT_SHADE_TAIL32): parity over the shading tests (one -k),
# then base vs the tail64 variant on the headline and the shipped light
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jit.py tests/test_gpu_parity.py \
    tests/test_gpu_stochastic.py -k "reference_canvas or dense_band or headline or benchmark_scene or row_sorted or lazy_ambient or cornell_gi_24 or cornell_shipped or cfg4 or goldens or math_core" \
    > gpurun_out/pytest_r06_p.log 2>&1 || { tail -30 gpurun_out/pytest_r06_p.log; exit 1; }
tail -2 gpurun_out/pytest_r06_p.log
bash tools/gpu_var.sh cornell_direct_1920x1080_8x8 r06_tail32 base tail64 base tail64 || exit 1
bash tools/gpu_var.sh cornell_shipped_1920x1080_8x8 r06_tail32_shipped base tail64 || exit 1
