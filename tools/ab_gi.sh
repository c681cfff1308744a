#!/bin/bash
# A/B timing of alternative device libraries (exp/<name>.so) on the GI scene at 480x270 (one frame
# each: photon pass + final gather), run via gpurun from the repo root
SC=${SC:-cornell_gi_480x270_8x8}
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
for lib in base "$@"; do
  if [ "$lib" = base ]; then cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; else cp variants/$lib.so fast_ray_tracer_amd/lib/libfrt_device.so; fi
  timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-render-multi --gi-steps 0 --scene $SC 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', 'ms/frame', d['ms_per_step'], 'gi', d['kernel_ms_per_frame'].get('gi'))" || { cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; exit 1; }
done
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
