#!/bin/bash
# Walk statistics (FRT_WALK_STATS build exp/stats.so) of one bench frame; run via gpurun from the repo root.
#   hipcc ... -DFRT_WALK_STATS -o exp/stats.so fast_ray_tracer_amd/csrc/frt_engine.hip   (build first, on the CPU)
SCENE=${1:-cornell_direct_800_4x4}
mkdir -p gpurun_out
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
cp exp/stats.so fast_ray_tracer_amd/lib/libfrt_device.so
timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --scene $SCENE > gpurun_out/stats_$SCENE.json 2> gpurun_out/stats_$SCENE.err
rc=$?
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
grep -E "walk stats|node visits|walk prof|prepare prof" gpurun_out/stats_$SCENE.err
exit $rc
