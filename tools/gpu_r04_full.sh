#!/bin/bash
# round 4: the whole -m gpu suite, then the headline A/B of the new JIT defaults against the previous ones
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_full.log
[ $rc -ne 0 ] && exit $rc
TESTS="" STEPS=5 bash tools/gpu_ab_env.sh defaults "FRT_JIT=1" "FRT_JIT_PART=17 FRT_JIT_SUB=0 FRT_JIT_TILE=32" "FRT_JIT=1"
