#!/bin/bash
# round 6, second pass: the row-ordered shading's modes and the node-major group size on the shipped frame; the GI
# estimate's phase split (variants/prof.so, -DFRT_WALK_PROF) on the 480x270 GI camera with the plain build's time beside it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "row_sorted" > gpurun_out/pytest_r06_b.log 2>&1 || { tail -30 gpurun_out/pytest_r06_b.log; exit 1; }
tail -2 gpurun_out/pytest_r06_b.log
bash tools/gpu_ab.sh cornell_shipped_1920x1080_8x8 r06_shipped_b "FRT_JIT_NODE_MAJOR=2" "FRT_JIT_NODE_MAJOR=4" \
    "FRT_JIT_NODE_MAJOR=8" "FRT_JIT_NODE_MAJOR=4 FRT_SHADE_STAGE=2" "FRT_JIT_NODE_MAJOR=4 FRT_SHADE_STAGE=1" \
    "FRT_JIT_NODE_MAJOR=4 FRT_SHADE_STAGE=0" || exit 1
B="--scene cornell_gi_480x270_8x8 --gi-steps 0 --shipped-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy --steps 1 --warmup 0"
timeout -k 10 300 python3 bench.py $B > gpurun_out/gi480_plain.json 2> gpurun_out/gi480_plain.err || exit 1
python3 tools/bench_brief.py gpurun_out/gi480_plain.json | head -3
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
cp variants/prof.so fast_ray_tracer_amd/lib/libfrt_device.so
timeout -k 10 600 python3 bench.py $B > gpurun_out/gi480_prof.json 2> gpurun_out/gi480_prof.err
rc=$?
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
[ $rc -ne 0 ] && { tail -5 gpurun_out/gi480_prof.err; exit $rc; }
grep "estimate prof" gpurun_out/gi480_prof.err | tail -1
