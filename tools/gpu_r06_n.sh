#!/bin/bash
# round 6: render_multi's pinned, pooled canvas (no staging copy, no page faults, no Python copy): its tests, then the
# drop-in timings (cold / warm / second process) and the headline frame at render_multi's batch (8 M) and the bench's
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "render_multi or drop_in" > gpurun_out/pytest_r06_n.log 2>&1 || { tail -30 gpurun_out/pytest_r06_n.log; exit 1; }
tail -2 gpurun_out/pytest_r06_n.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --gi-steps 0 --shipped-steps 0 --no-cpu-baseline \
    --no-scaling-proxy > gpurun_out/bench_r06_rm.json 2> gpurun_out/bench_r06_rm.err || { tail -20 gpurun_out/bench_r06_rm.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r06_rm.json').read().splitlines()[-1])
print('frame', d['ms_per_step']); [print(k, d[k]) for k in d if k.startswith('render_multi')]" | tee gpurun_out/rm_r06.txt
for b in 8388608 33554432 134217728; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --gi-steps 0 --shipped-steps 0 --no-cpu-baseline --no-render-multi \
      --no-scaling-proxy --batch-samples $b > gpurun_out/bench_r06_b$b.json 2>> gpurun_out/bench_r06_rm.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('batch', sys.argv[2], 'frame ms', d['ms_per_step'], d['kernel_ms_per_frame'])" \
      gpurun_out/bench_r06_b$b.json $b | tee -a gpurun_out/rm_r06.txt
done
