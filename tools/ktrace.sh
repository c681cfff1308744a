#!/bin/bash
# Kernel trace of one bench frame (run via gpurun from the repo root): per-dispatch durations
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ktrace_${1:-x}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$OUT" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[-80:]:
    n = r["Kernel_Name"].split("(")[0][:40]
    print("%-40s grid=%9s start=%9.3f ms dur=%8.3f ms" % (n, r.get("Grid_Size_X", r.get("Grid_Size", "?")),
          (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
PY
