#!/bin/bash
# cfg4 stand-in (bounding_boxes_800x1000_4x4: 6 dragons, BVH, generic walk) profiles, run via gpurun from
# the repo root: the bench line, rocprof kernel-trace stats, PMC passes of k_trace and k_shadow.
# Summaries: gpurun_out/prof_TAG/pmc_<kernel>.json (tools/pmc_summary.py)
set -o pipefail
TAG=${1:-cfg4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
SC=bounding_boxes_800x1000_4x4
B="--steps 1 --warmup 0 --gi-steps 0 --no-cpu-baseline --no-render-multi --scene $SC"
mkdir -p "$OUT"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi --scene $SC > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- python3 "$R/bench.py" $B > "$OUT/kt.json" 2> "$OUT/kt.err" || exit $?
pmc() {  # dir kernel-regex counters...
    local d=$1 kre=$2; shift 2
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" $B > "$OUT/$(basename $d).json" 2> "$OUT/$(basename $d).err"
}
for K in k_trace k_shadow; do
    mkdir -p "$OUT/$K"
    pmc $K/sq "$K<" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
    pmc $K/mem "$K<" SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES || exit $?
    pmc $K/fetch "$K<" FETCH_SIZE || exit $?
    pmc $K/write "$K<" WRITE_SIZE || exit $?
done
cd "$R"
for K in k_trace k_shadow; do
    cp -r "$OUT/kt" "$OUT/$K/kt"
    python3 tools/pmc_summary.py "$OUT/$K" "$K<" $SC > "$OUT/pmc_$K.json" || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
d = json.loads(open(out + "/bench.json").read().strip().splitlines()[-1])
print("ms/frame", d["ms_per_step"], "value", d["value"], d.get("kernel_ms_per_frame"))
for f in glob.glob(out + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:10]:
        print("%-60s calls=%5s total=%9.2f ms avg=%8.3f ms %s%%" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"])/1e6, float(r["AverageNs"])/1e6, r["Percentage"]))
for k in ("k_trace", "k_shadow"):
    t = json.load(open(out + "/pmc_%s.json" % k))
    print(k, {kk: round(v, 3) if isinstance(v, float) else v for kk, v in t.items() if "frac" in kk or "per_wave" in kk or "bytes" in kk})
PY
