#!/bin/bash
# round 6 (late): the sum passes' record prefetch (FRT_SUM_TOUCH) — the estimate's GPU tests, then A/B on the 480x270
# GI camera against variants/notouch.so (tools/gpu_gi_var.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_photon_map.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "estimate or gather or photon" > gpurun_out/pytest_touch.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_touch.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_gi_var.sh touch base notouch base notouch || exit 1
cat gpurun_out/gi_ab_touch.txt
