#!/bin/bash
# round 4: one lane's closest-hit walk printed (FRT_JIT_TRACE_DBG) on a small frame (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
FRT_JIT_TRACE_STATS=1 FRT_JIT_TRACE_DBG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-render-multi --gi-steps 0 --scene cornell_direct_1920x1080_8x8 > gpurun_out/trace_dbg.log 2>&1
rc=$?
grep -a "frt_jit_trace" gpurun_out/trace_dbg.log | head -60
exit $rc
