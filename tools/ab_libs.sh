#!/bin/bash
# A/B timing of alternative device libraries (exp/<name>.so), run via gpurun from the repo root
FLAGS=${FLAGS:-0}
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
for lib in base "$@"; do
  if [ "$lib" = base ]; then cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; else cp exp/$lib.so fast_ray_tracer_amd/lib/libfrt_device.so; fi
  FRT_WALK_FLAGS=$FLAGS timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', 'ms/frame', d['ms_per_step'], 'shadow', d['kernel_ms_per_frame']['shadow'])" || exit 1
done
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
