#!/bin/bash
# -m gpu tests, one headline bench line (no GI / CPU legs) and the pair kernel's statistics (run via gpurun)
#   tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1])
print('%.2f ms/frame' % d['ms_per_step'], {k: round(v, 1) for k, v in d['kernel_ms_per_frame'].items()}, d['shadow_pass']['kernels_ms_per_frame'], d['shadow_pass']['shadow_rays_walked_per_ray'])"
FRT_JIT_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --gi-steps 0 --no-cpu-baseline --no-render-multi > gpurun_out/jstats_$TAG.json 2> gpurun_out/jstats_$TAG.err || exit $?
grep "jit stats" gpurun_out/jstats_$TAG.err | head -20
