#!/bin/bash
# round 6, fifth pass: the beam stages' wave-summed run counts (FRT_JIT_RUN_COUNTS) — stage parity tests, then
# headline and shipped A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_jit.py -k "headline or tile_and_sub or shipped or equals_generic or split or production_default" \
    > gpurun_out/pytest_r06_e.log 2>&1 || { tail -30 gpurun_out/pytest_r06_e.log; exit 1; }
tail -2 gpurun_out/pytest_r06_e.log
bash tools/gpu_ab.sh cornell_direct_1920x1080_8x8 r06_runcounts "FRT_JIT_RUN_COUNTS=0" "FRT_X=1" "FRT_JIT_RUN_COUNTS=0" "FRT_X=1" || exit 1
bash tools/gpu_ab.sh cornell_shipped_1920x1080_8x8 r06_runcounts_shipped "FRT_JIT_RUN_COUNTS=0" "FRT_X=1"
