#!/bin/bash
# A/B of environment knobs on one scene (one frame each; run via gpurun from the repo root)
#   SC=scene tools/ab_env.sh "FRT_GATHER_SORT=0" "FRT_GATHER_SORT=1" ...
SC=${SC:-cornell_gi_480x270_8x8}
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --steps ${STEPS:-1} --warmup ${WARMUP:-0} --no-cpu-baseline --no-render-multi --gi-steps 0 --scene $SC 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', 'ms/frame', d['ms_per_step'], d['kernel_ms_per_frame'], d.get('sub_ms_per_frame', ''))" || exit 1
done
