#!/bin/bash
# A/B of the photon grid's cell size and cell budget (FRT_PM_CELL_DIV cells per radius,
# FRT_PM_MAX_CELLS_LOG2) on a GI scene (run via gpurun from the repo root)
#   tools/ab_grid.sh "3:24 3:26 4:27" [scene]
SC=${2:-cornell_gi_480x270_8x8}
for v in $1; do
  dv=${v%%:*}; mc=${v##*:}
  FRT_PM_CELL_DIV=$dv FRT_PM_MAX_CELLS_LOG2=$mc timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-render-multi --gi-steps 0 --scene $SC 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('div $dv cells 2^$mc', 'ms/frame', d['ms_per_step'], d['kernel_ms_per_frame'], {k: v for k, v in d.items() if 'photon' in k or 'gather' in k})" || exit 1
done
