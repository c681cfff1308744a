#!/bin/bash
# round 4: fused shading terms + pow_ns without the first product: parity tests, then the headline (bench settings)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_shade2.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_shade2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --gi-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy > gpurun_out/bench_shade2.json 2>/dev/null && tail -1 gpurun_out/bench_shade2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms', d['ms_per_step'], {k: round(v, 2) for k, v in d['kernel_ms_per_frame'].items()}, {k: round(v, 2) for k, v in d.get('sub_ms_per_frame', {}).items()})"
