#!/bin/bash
# Profile the bench workload on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats           -> per-kernel average durations
#   2. --pmc FETCH_SIZE, --pmc WRITE_SIZE          -> HBM-side traffic of the dominant (shadow) kernel, one pass each
#   3. --pmc SQ_* VALU / wave counters, GRBM       -> VALU issue utilisation of the same kernel
# Output under gpurun_out/prof_<tag>/; tools/profile_summary.py turns it into the profiles/ JSON.
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
KRE=${KREGEX:-frt_jit_shadow}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
STEPS=${STEPS:-3}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup 1 --no-cpu-baseline > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit $?
pass() {  # name, counters...
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d "$OUT/$name" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err"
}
pass fetch FETCH_SIZE || exit $?
pass write WRITE_SIZE || exit $?
pass valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 || exit $?
pass clock GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
python3 "$R/tools/profile_summary.py" "$OUT" "$KRE"
