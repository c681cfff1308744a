#!/bin/bash
# GPU parity tests + a short bench (run via gpurun from the repo root). Usage: tools/gpu_check.sh TAG [bench args]
set -o pipefail
TAG=${1:-chk}; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
tail -1 gpurun_out/bench_$TAG.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('ms/frame', d['ms_per_step'], 'Mrays/s', d['value'], d['kernel_ms_per_frame'])"
