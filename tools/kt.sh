#!/bin/bash
# rocprofv3 kernel trace + stats of a bench workload, no PMC (tools/kt.sh TAG SCENE [extra bench args]);
# prints the per-kernel table (calls, average and total ms) into gpurun_out/kt_TAG.txt
set -o pipefail
TAG=$1; SC=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/kt_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- \
    python3 "$R/bench.py" --scene $SC --steps 3 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi \
    --no-scaling-proxy --shipped-steps 0 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cd "$R"
python3 - "$OUT" > gpurun_out/kt_$TAG.txt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = 0
for r in rows:
    tot += int(r["Calls"])
    print("%-70s %5s %9.3f %9.3f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
print("total calls", tot)
PY
cat gpurun_out/kt_$TAG.txt
