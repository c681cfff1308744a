#!/bin/bash
# round 6: parity after the closest-hit deferral and the child halves (one -k over the files: pytest applies the last
# -k to every file): closest hit vs the generic walk, goldens, headline rows / band / split, lazy ambient, gather order,
# GI and shipped statistical gates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jit.py tests/test_gpu_parity.py \
    tests/test_gpu_stochastic.py -k "closest_hit or equals_generic or reference_canvas or headline or benchmark_scene or lazy_ambient or gather or cornell_gi_24 or cornell_shipped or cfg4 or mesh_search" \
    > gpurun_out/pytest_r06_l.log 2>&1 || { tail -30 gpurun_out/pytest_r06_l.log; exit 1; }
tail -2 gpurun_out/pytest_r06_l.log
