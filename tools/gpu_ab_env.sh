#!/bin/bash
# The JIT / parity tests that must stay bit-identical, then an A/B of environment knobs on the headline
# (run via gpurun from the repo root):   TESTS="tests/test_jit.py" tools/gpu_ab_env.sh TAG "A=0" "A=1" ...
set -o pipefail
TAG=${1:-abe}; shift
mkdir -p gpurun_out
if [ -n "${TESTS-tests/test_jit.py}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS-tests/test_jit.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
SC=${SC:-cornell_direct_1920x1080_8x8}
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup ${WARMUP:-1} --no-cpu-baseline --no-render-multi --gi-steps 0 --scene $SC 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', 'ms/frame', d['ms_per_step'], {k: round(v, 2) for k, v in d['kernel_ms_per_frame'].items()}, {k: round(v, 2) for k, v in d.get('sub_ms_per_frame', {}).items()}, d['shadow_pass']['shadow_rays_walked_per_ray'])" | tee -a gpurun_out/ab_$TAG.txt || exit 1
done
