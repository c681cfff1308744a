#!/bin/bash
# A/B of the photon grid's cell size (FRT_PM_CELL_DIV cells per radius) on cornell_gi_480x270_8x8
SC=${SC:-cornell_gi_480x270_8x8}
for dv in 3 4 5 2; do
  FRT_PM_CELL_DIV=$dv timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-render-multi --gi-steps 0 --scene $SC 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cell r/$dv', 'ms/frame', d['ms_per_step'], 'gi', d['kernel_ms_per_frame'].get('gi'))" || exit 1
done
