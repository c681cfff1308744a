#!/bin/bash
# Kernel trace of one headline frame (run via gpurun from the repo root): total time per (kernel, grid size),
# i.e. per wavefront level (level 0 of the headline batches has 2^21 samples), to see which level of which kernel
# the frame's time goes to.  tools/ktrace_levels.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}; shift
OUT=$R/gpurun_out/ktl_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 \
    --gi-steps 0 --no-cpu-baseline --no-render-multi "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 - "$OUT" <<'PY' | tee "$OUT/levels.txt"
import collections, csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    k = (r["Kernel_Name"].split("(")[0].replace("void ", "")[:34], int(r.get("Grid_Size_X", r.get("Grid_Size", 0))))
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
tot = sum(v[1] for v in agg.values())
for (n, g), (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print("%-34s grid=%10d calls=%5d total=%9.3f ms (%5.1f %%)" % (n, g, c, ms, 100 * ms / tot))
print("all kernels: %.3f ms" % tot)
PY
