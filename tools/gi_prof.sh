#!/bin/bash
# The estimate's phase profile (variants/prof.so: -DFRT_WALK_PROF) on a GI scene (run via gpurun from the repo root)
SC=${SC:-cornell_gi_480x270_8x8}
mkdir -p gpurun_out
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
cp variants/${1:-prof}.so fast_ray_tracer_amd/lib/libfrt_device.so
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-render-multi --gi-steps 0 --scene $SC > gpurun_out/gi_prof.json 2> gpurun_out/gi_prof.err
rc=$?
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
grep -E "estimate prof" gpurun_out/gi_prof.err | tail -1
exit $rc
