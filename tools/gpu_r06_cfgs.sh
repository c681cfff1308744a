#!/bin/bash
# round 6: cfg3 / cfg4 bench lines (bench.py --scene, GI / shipped / proxies / render_multi / CPU baseline off)
set -o pipefail
mkdir -p gpurun_out
for sc in cornell_direct_800_4x4 bounding_boxes_800x1000_4x4; do
  timeout -k 10 300 python -u bench.py --scene $sc --steps 10 --warmup 2 --gi-steps 0 --shipped-steps 0 --no-cpu-baseline \
      --no-render-multi --no-scaling-proxy > gpurun_out/bench_r06_$sc.json 2> gpurun_out/bench_r06_$sc.err || exit $?
  tail -1 gpurun_out/bench_r06_$sc.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc', d['ms_per_step'], d['kernel_ms_per_frame'])"
done
