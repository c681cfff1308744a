#!/bin/bash
# round 4: the headline bench line without the slow extras (roofline blocks), then cfg3 and cfg4 bench lines
set -o pipefail
mkdir -p gpurun_out
B="--gi-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 $B > gpurun_out/bench_roof.json 2> gpurun_out/bench_roof.err && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 $B --scene cornell_direct_800_4x4 > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 $B --scene bounding_boxes_800x1000_4x4 > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err
