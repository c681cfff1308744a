#!/bin/bash
# the whole round-end check: the whole -m gpu suite, smoke(), then the default bench line (headline, shipped, GI, proxies, render_multi,
# CPU baseline):   tools/gpu_full.sh TAG
TAG=${1:-r06}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}_full.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_${TAG}_full.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.txt 2>&1 || { tail -5 gpurun_out/smoke_${TAG}.txt; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.txt
timeout -k 10 900 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
tail -1 gpurun_out/bench_${TAG}.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms', d['ms_per_step'], 'value', d['value'], 'shipped', d.get('shipped', {}).get('ms_per_step'), 'gi', d.get('gi', {}).get('ms_per_step'), 'gi shadow', d.get('gi', {}).get('kernel_ms_per_frame', {}).get('shadow')); print('rm', {k: v for k, v in d.items() if k.startswith('render_multi_wall')}); print('proxy', json.dumps(d.get('scaling_proxy'))[:300])"
