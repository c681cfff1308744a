#!/bin/bash
# One GPU round trip (run via gpurun from the repo root): -m gpu tests, smoke, the default bench line.
#   tools/gpu_round.sh TAG [bench args]
set -o pipefail
TAG=${1:-chk}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || exit $?
cat gpurun_out/smoke_$TAG.txt
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
tail -1 gpurun_out/bench_$TAG.json
