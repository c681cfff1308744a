#!/bin/bash
# One-frame bench of other BASELINE configs (run via gpurun from the repo root): tools/bench_scenes.sh SCENE...
mkdir -p gpurun_out
for sc in "$@"; do
  timeout -k 10 ${TMO:-300} python bench.py --steps ${STEPS:-1} --warmup ${WARMUP:-0} --no-cpu-baseline --scene $sc > gpurun_out/bench_$sc.json 2> gpurun_out/bench_$sc.err
  rc=$?
  [ $rc -ne 0 ] && { echo "$sc rc=$rc"; tail -5 gpurun_out/bench_$sc.err; exit $rc; }
  tail -1 gpurun_out/bench_$sc.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc', 'ms/frame', d['ms_per_step'], 'Mrays/s', d['value'], d['kernel_ms_per_frame'])"
done
