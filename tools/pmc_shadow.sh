#!/bin/bash
# PMC passes over the k_shadow launches of one bench frame (run via gpurun from the repo root).
#   tools/pmc_shadow.sh TAG "CTR1 CTR2 ..." ["CTR ..."]   one rocprofv3 pass per quoted set
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
k=0
for set in "$@"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "${KREGEX:-k_shadow}" -f csv -d "$OUT/p$k" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/p$k.json" 2> "$OUT/p$k.err" || exit $?
done
python3 "$R/tools/pmc_sum.py" "$OUT"
