#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench (headline frames + one GI frame), run via gpurun
# from the repo root. Output: gpurun_out/prof_TAG/kt/**/run_kernel_stats.csv
set -o pipefail
TAG=${1:-kt}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --gi-steps 1 --no-cpu-baseline --no-render-multi > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:12]:
        print("%-60s calls=%5s total=%10.2f ms avg=%8.3f ms %s%%" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"])/1e6, float(r["AverageNs"])/1e6, r["Percentage"]))
PY
