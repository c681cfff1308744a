#!/bin/bash
# round 6, third pass: parity of the one-range level 0 and the statistics-only counters (headline rows, dense band,
# split invariance, the stage tests); GI estimate builds; the one-range level 0 and node-major lanes on the headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "headline or benchmark_scene or cfg4" tests/test_jit.py -k "headline or split or tile_and_sub" \
    > gpurun_out/pytest_r06_c.log 2>&1 || { tail -30 gpurun_out/pytest_r06_c.log; exit 1; }
tail -2 gpurun_out/pytest_r06_c.log
bash tools/gpu_ab.sh cornell_direct_1920x1080_8x8 r06_headline_range "FRT_JIT_MAX_PAIRS=268435455" "FRT_X=0" \
    "FRT_JIT_NODE_MAJOR=4" "FRT_JIT_MAX_PAIRS=268435455" "FRT_X=0" || exit 1
bash tools/gpu_gi_var.sh r06_est base scan2 scan4 sqrt1 w3 base || exit 1
bash tools/gpu_ab.sh cornell_shipped_1920x1080_8x8 r06_shipped_defaults "FRT_X=0"
