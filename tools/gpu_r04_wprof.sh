#!/bin/bash
# round 4: k_prepare's cycle split (FRT_WALK_PROF variant: ray, hit load, prepare, spawn, stores) on one headline
# frame (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
cp variants/wprof.so fast_ray_tracer_amd/lib/libfrt_device.so
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --gi-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy > gpurun_out/wprof.json 2> gpurun_out/wprof.err
rc=$?
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
grep -a "prepare prof" gpurun_out/wprof.err | tail -2
exit $rc
