#!/bin/bash
# round 6: closest-hit CSG units with the open entry orders settled after the first positive entry — bit-identity to
# the generic walk (test_jit_closest_hit_equals_generic_walk), goldens, headline rows; the undecided count; headline A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_jit.py -k "closest_hit or equals_generic" tests/test_gpu_parity.py -k "reference_canvas or headline or benchmark_scene or cfg4" \
    > gpurun_out/pytest_r06_j.log 2>&1 || { tail -30 gpurun_out/pytest_r06_j.log; exit 1; }
tail -2 gpurun_out/pytest_r06_j.log
timeout -k 10 300 python3 tools/trace_redo_dump.py cornell_direct_1920x1080_8x8 gpurun_out/trace_redo2.npy > gpurun_out/trace_redo2.txt 2>&1 || exit 1
grep "generic walk\|undecided" gpurun_out/trace_redo2.txt
bash tools/gpu_ab.sh cornell_direct_1920x1080_8x8 r06_trace_defer "FRT_X=0" "FRT_X=1"
