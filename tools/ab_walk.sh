#!/bin/bash
# A/B timing of walk variants selected by FRT_WALK_FLAGS (run via gpurun from the repo root)
for f in "$@"; do
  FRT_WALK_FLAGS=$f timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('flags=$f', 'ms/frame', d['ms_per_step'], 'shadow', d['kernel_ms_per_frame']['shadow'])" || exit 1
done
