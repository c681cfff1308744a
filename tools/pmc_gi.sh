#!/bin/bash
# Kernel stats + SQ counters of the final-gather kernel on the GI workload (run via gpurun from the repo root)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
SC=${SC:-cornell_gi_480x270_8x8}
KRE=${KRE:-k_gather_shade}
OUT=$R/gpurun_out/pmc_gi_${TAG:-a}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d "$OUT/$name" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --scene $SC > "$OUT/$name.json" 2> "$OUT/$name.err"
}
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --scene $SC > "$OUT/kt.json" 2> "$OUT/kt.err" &&
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA &&
run b SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VALU_FMA_F64 || exit $?
python3 - "$OUT" "$KRE" <<'PY'
import csv, glob, re, sys, collections
out, kre = sys.argv[1], sys.argv[2]
for f in glob.glob(out + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:12]:
        print("%-70s calls=%5s total=%9.2f ms avg=%8.3f ms %s%%" % (r["Name"][:70], r["Calls"], float(r["TotalDurationNs"])/1e6, float(r["AverageNs"])/1e6, r["Percentage"]))
tot = collections.defaultdict(float)
for f in glob.glob(out + "/[ab]/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if re.search(kre, r["Kernel_Name"]): tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()): print("%-28s %.4g" % (k, v))
PY
