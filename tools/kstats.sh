#!/bin/bash
# rocprofv3 --kernel-trace --stats of one bench frame of a scene (run via gpurun from the repo root)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
SC=${1:-cornell_direct_800_4x4}
OUT=$R/gpurun_out/kstats_$SC
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${TMO:-300} rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- python3 "$R/bench.py" --steps ${STEPS:-1} --warmup ${WARMUP:-0} --no-cpu-baseline --scene $SC ${KS_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:25]: print('%-60s calls=%6s total=%10.3f ms avg=%9.4f ms %6s%%' % (r['Name'][:60], r['Calls'], float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e6, r['Percentage']))
"
