#!/bin/bash
# Photon-estimate round trip (run via gpurun from the repo root; build exp/prof.so first with
#   hipcc ... -DFRT_WALK_PROF -o exp/prof.so frt_engine.hip frt_jit.hip):
# photon-map + GI parity tests, the estimate's phase profile on cornell_gi_480x270_8x8, the GI bench line.
#   tools/gi_round.sh TAG
set -o pipefail
TAG=${1:-gi}
SC=cornell_gi_480x270_8x8
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_photon_map.py tests/test_gpu_stochastic.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gi_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gi_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gi_tests_$TAG.log
if [ -f exp/prof.so ]; then
  cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
  cp exp/prof.so fast_ray_tracer_amd/lib/libfrt_device.so
  timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-render-multi --gi-steps 0 --scene $SC > gpurun_out/gi_prof_$TAG.json 2> gpurun_out/gi_prof_$TAG.err
  rc=$?
  cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
  grep -E "estimate prof" gpurun_out/gi_prof_$TAG.err | tail -1
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-render-multi --gi-steps 0 --scene $SC > gpurun_out/gi_bench_$TAG.json 2> gpurun_out/gi_bench_$TAG.err || exit $?
python - "$TAG" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/gi_bench_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
print("480x270 GI frame ms", d["ms_per_step"], "kernel_ms", d.get("kernel_ms_per_frame"))
PY
