#!/bin/bash
# round 4: FRT_JIT_STATS pair / ray counts of one headline frame under several settings (stderr of bench.py)
set -o pipefail
mkdir -p gpurun_out
for e in "$@"; do
  tag=$(echo "$e" | tr ' =' '_-')
  env FRT_JIT_STATS=1 $e timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy --gi-steps 0 > gpurun_out/stats_$tag.json 2> gpurun_out/stats_$tag.err || exit $?
  grep "frt jit stats" gpurun_out/stats_$tag.err | grep -v "node \|site" | sed "s/^/$e: /"
done
