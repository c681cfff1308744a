#!/bin/bash
# Profile the bench workload on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats  -> per-kernel average durations
#   2. --pmc FETCH_SIZE / MemWrites32B   -> HBM-side traffic per dispatch (one pass each:
#      gfx950 cannot collect FETCH_SIZE with another memory counter; WRITE_SIZE is absent)
#   3. --pmc FP64 VALU instruction counts (own pass; optional)
# Output under gpurun_out/prof_<tag>/ ; summaries are copied into profiles/ by hand.
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
STEPS=${STEPS:-3}
timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup 1 --no-cpu-baseline > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" &&
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_fetch_bench.json" 2> "$OUT/pmc_fetch.err" &&
timeout -k 10 200 rocprofv3 --pmc MemWrites32B -f csv -d "$OUT/pmc_write" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_write_bench.json" 2> "$OUT/pmc_write.err" &&
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -f csv \
    -d "$OUT/pmc_f64" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_f64_bench.json" 2> "$OUT/pmc_f64.err"
rc=$?
find "$OUT" -name "*.csv" | head -50
exit $rc
