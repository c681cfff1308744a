#!/bin/bash
# Occupancy A/B of the scene-specialised shadow kernels on the headline frame (run via gpurun):
#   tools/ab_waves.sh "SHADOW_WAVES:BEAM_WAVES" ...   (0 = the compiler's choice)
mkdir -p gpurun_out
for wb in "$@"; do
  w=${wb%%:*}; b=${wb##*:}
  FRT_JIT_WAVES=$w FRT_JIT_BEAM_WAVES=$b timeout -k 10 300 python bench.py --steps 3 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('waves %s: %8.2f ms/frame' % ('$wb', d['ms_per_step']), d['shadow_pass']['kernels_ms_per_frame'])" || exit 1
done
