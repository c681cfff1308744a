#!/bin/bash
# -m gpu tests, then the per-level kernel trace of one headline frame (run via gpurun from the repo root)
#   tools/gpu_ab.sh TAG [bench args]
set -o pipefail
TAG=${1:-ab}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/ktrace_levels.sh $TAG "$@"
