#!/bin/bash
# A/B timing of alternative device libraries (variants/<name>.so; "base" = the built one) on one scene
# (run via gpurun from the repo root):   SC=scene STEPS=k tools/ab_lib.sh name ...
SC=${SC:-cornell_direct_1920x1080_8x8}
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
for lib in base "$@"; do
  if [ "$lib" = base ]; then cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; else cp variants/$lib.so fast_ray_tracer_amd/lib/libfrt_device.so; fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup ${WARMUP:-1} --no-cpu-baseline --no-render-multi --gi-steps 0 --scene $SC 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', 'ms/frame', d['ms_per_step'], d['kernel_ms_per_frame'], d.get('sub_ms_per_frame', ''))" || { cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; exit 1; }
done
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
