#!/bin/bash
# round 6: k_prepare's phase split on the headline frame (variants/prof.so, -DFRT_WALK_PROF: s_memtime stamps)
set -o pipefail
mkdir -p gpurun_out
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
cp variants/prof.so fast_ray_tracer_amd/lib/libfrt_device.so
timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --gi-steps 0 --shipped-steps 0 --no-cpu-baseline --no-render-multi \
    --no-scaling-proxy > gpurun_out/prof_headline.json 2> gpurun_out/prof_headline.err
rc=$?
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
[ $rc -ne 0 ] && { tail -5 gpurun_out/prof_headline.err; exit $rc; }
grep "prepare prof" gpurun_out/prof_headline.err | tail -1
