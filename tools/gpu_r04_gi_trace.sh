#!/bin/bash
# round 4: the GI frame with the generic closest-hit walk and with frt_jit_trace (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --steps 1 --warmup 0 --gi-steps 1 --no-cpu-baseline --no-render-multi --no-scaling-proxy 2>gpurun_out/gi_trace.err | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['gi']; print('$e', 'gi ms', g['ms_per_step'], g['kernel_ms_per_frame'], g.get('gather_est'))" | tee -a gpurun_out/ab_gi_trace.txt || exit 1
done
