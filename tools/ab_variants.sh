#!/bin/bash
# A/B of device-library variants (variants/<name>.so from tools/build_variant.sh) on the headline and the cfg4
# stand-in (run via gpurun from the repo root):   tools/ab_variants.sh NAME...
set -o pipefail
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
for lib in base "$@" base; do
  if [ "$lib" = base ]; then cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; else cp variants/$lib.so fast_ray_tracer_amd/lib/libfrt_device.so; fi
  for SC in ${SCENES:-cornell_direct_1920x1080_8x8 bounding_boxes_800x1000_4x4}; do
    timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi --scene $SC 2>/dev/null | tail -1 | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', '$SC', 'ms/frame', d['ms_per_step'], {k: round(v, 2) for k, v in d['kernel_ms_per_frame'].items()})" || { cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; exit 1; }
  done
done
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
