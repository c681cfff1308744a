#!/bin/bash
# round 6 (late): the per-frame gather knobs (FRT_GATHER_SORT / FRT_GATHER_JIT read per chunk) — the gather tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "gather" > gpurun_out/pytest_gather_knobs.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_gather_knobs.log | tail -6; exit $rc
