#!/bin/bash
# A/B of the samples per batch on the headline frame (run via gpurun from the repo root): tools/ab_batch.sh N...
set -o pipefail
mkdir -p gpurun_out
for b in "$@"; do
    timeout -k 10 240 python -u bench.py --steps 4 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy \
        --batch-samples $b > gpurun_out/ab_batch_$b.json 2> gpurun_out/ab_batch_$b.err || exit $?
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_batch_$b.json').read().strip().splitlines()[-1])
print('batch %10d: %8.2f ms/frame' % ($b, d['ms_per_step']), {k: round(v, 1) for k, v in d['kernel_ms_per_frame'].items()})"
done
