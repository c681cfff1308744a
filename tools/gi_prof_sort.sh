#!/bin/bash
# round 5: the estimate's phase cycles (variants/prof.so, -DFRT_WALK_PROF) on cornell_gi_480x270_8x8 with the
# gather requests in gather order and sorted: tools/gi_prof_sort.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gi_prof_sort
mkdir -p "$OUT"
cp "$R/fast_ray_tracer_amd/lib/libfrt_device.so" /tmp/frt_base.so
cp "$R/variants/prof.so" "$R/fast_ray_tracer_amd/lib/libfrt_device.so"
rc=0
for mode in 0 -1; do
  FRT_GATHER_SORT=$mode timeout -k 10 300 python3 "$R/bench.py" --scene cornell_gi_480x270_8x8 --gi-steps 0 --no-cpu-baseline \
      --no-render-multi --no-scaling-proxy --shipped-steps 0 --steps 1 --warmup 0 > "$OUT/prof$mode.json" 2> "$OUT/prof$mode.err" || { rc=$?; break; }
  echo "FRT_GATHER_SORT=$mode"; grep "estimate prof" "$OUT/prof$mode.err" | tail -1
done
cp /tmp/frt_base.so "$R/fast_ray_tracer_amd/lib/libfrt_device.so"
exit $rc
