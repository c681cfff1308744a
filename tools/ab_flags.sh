#!/bin/bash
# A/B timing of FRT_WALK_FLAGS experiment bits (run via gpurun from the repo root): per-kernel ms per frame
mkdir -p gpurun_out
for f in "$@"; do
  FRT_WALK_FLAGS=$f timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$f.json 2> gpurun_out/ab_$f.err
  rc=$?
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && { echo "flags=$f rc=$rc (stop)"; exit $rc; }
  tail -1 gpurun_out/ab_$f.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('flags=$f', 'ms/frame', d['ms_per_step'], d['kernel_ms_per_frame'])" || { echo "flags=$f rc=$rc"; tail -3 gpurun_out/ab_$f.err; }
done
