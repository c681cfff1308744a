#!/bin/bash
# round 4: shading algebra (FRT_SHADE_ALG): the parity tests, the headline, then the samples-per-batch A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stochastic.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_shade.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_shade.log
[ $rc -ne 0 ] && exit $rc
TESTS="" STEPS=5 bash tools/gpu_ab_env.sh shade "FRT_JIT=1" && bash tools/ab_batch.sh 8388608 33554432 134217728
