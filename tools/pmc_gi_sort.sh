#!/bin/bash
# round 5: k_gather_est's L2 hits/misses and fabric bytes with the requests in gather order (FRT_GATHER_SORT=0) and
# sorted (default), one GI frame per PMC pass: SC=<scene> tools/pmc_gi_sort.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gi_sort
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SC=${SC:-cornell_gi_480x270_8x8}
for mode in 0 -1; do
  export FRT_GATHER_SORT=$mode
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gather_est -f csv -d "$OUT/fetch$mode" -o run -- \
      python3 "$R/tools/gi_frame.py" $SC > "$OUT/fetch$mode.txt" 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-include-regex k_gather_est -f csv -d "$OUT/tcc$mode" -o run -- \
      python3 "$R/tools/gi_frame.py" $SC > "$OUT/tcc$mode.txt" 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-include-regex k_gather_est -f csv -d "$OUT/tcp$mode" -o run -- \
      python3 "$R/tools/gi_frame.py" $SC > "$OUT/tcp$mode.txt" 2>&1 || exit $?
done
cd "$R" && for d in "$OUT"/*/; do echo "== $d"; python3 tools/pmc_sum.py "$d"; done > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
