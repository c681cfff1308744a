#!/bin/bash
# Light part size A/B on the headline frame (run via gpurun): tools/ab_parts2.sh SIZES...
mkdir -p gpurun_out
for ps in "$@"; do
  FRT_JIT_PART=$ps timeout -k 10 300 python bench.py --steps 3 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('part %3d: %8.2f ms/frame' % ($ps, d['ms_per_step']), d['shadow_pass']['kernels_ms_per_frame'], d['shadow_pass']['shadow_rays_walked_per_ray'])" || exit 1
done
