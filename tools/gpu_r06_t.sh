#!/bin/bash
# round 6 (late): the one-reciprocal BRDF factor (FRT_SHADE_MERGE) — shading parity tests, A/B on the headline and
# the shipped light against variants/nomerge.so, and k_gather_est's phase split (variants/prof.so, -DFRT_WALK_PROF:
# s_memtime stamps) on cornell_gi_480x270_8x8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "reference_canvas or headline_rows or dense_band or math_core or row_sorted or shipped" > gpurun_out/pytest_merge.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_merge.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_var.sh cornell_direct_1920x1080_8x8 merge_head base nomerge base || exit 1
bash tools/gpu_var.sh cornell_shipped_1920x1080_8x8 merge_ship base nomerge || exit 1
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
cp variants/prof.so fast_ray_tracer_amd/lib/libfrt_device.so
FRT_STATS_OUT=1 timeout -k 10 300 python3 tools/gi_frame.py cornell_gi_480x270_8x8 > gpurun_out/gi_prof.txt 2> gpurun_out/gi_prof.err
rc=$?
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
[ $rc -ne 0 ] && { tail -5 gpurun_out/gi_prof.err; exit $rc; }
grep -a "estimate prof" gpurun_out/gi_prof.err | tail -2
cat gpurun_out/ab_merge_head_all.txt gpurun_out/ab_merge_ship_all.txt
