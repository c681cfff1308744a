#!/bin/bash
# round 4: the default bench line (headline, GI, proxies, render_multi, CPU baseline) and smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r04.json 2> gpurun_out/bench_r04.err || { tail -20 gpurun_out/bench_r04.err; exit 1; }
tail -1 gpurun_out/bench_r04.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms', d['ms_per_step'], 'value', d['value'], 'gi', d.get('gi', {}).get('ms_per_step'), 'proxy', json.dumps(d.get('scaling_proxy'))[:400]); print('rm', {k: v for k, v in d.items() if k.startswith('render_multi')})" | cut -c1-1500
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
