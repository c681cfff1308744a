#!/bin/bash
# round 5: multi-row beam hierarchy — the JIT parity tests, then the shipped and headline frames
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_jit.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_jit.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_r05_jit.log
[ $rc -ne 0 ] && exit $rc
for sc in cornell_shipped_1920x1080_8x8 cornell_direct_1920x1080_8x8; do
  timeout -k 10 300 python -u bench.py --scene $sc --steps 5 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi \
    --no-scaling-proxy > gpurun_out/bench_r05_$sc.json 2> gpurun_out/bench_r05_$sc.err || { tail -20 gpurun_out/bench_r05_$sc.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], 'ms', d['ms_per_step'], json.dumps(d['kernel_ms_per_frame']), json.dumps(d['shadow_pass']['kernels_ms_per_frame']))" gpurun_out/bench_r05_$sc.json
done
