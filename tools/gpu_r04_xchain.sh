#!/bin/bash
# round 4: transform chains from one table (xf_chain): the GPU parity / JIT tests, then the headline frame
# (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_powbits.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_powbits.log
[ $rc -ne 0 ] && exit $rc
STEPS=3 TESTS= bash tools/gpu_ab_env.sh powbits "FRT_JIT_TRACE=1"
