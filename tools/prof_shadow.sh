#!/bin/bash
# rocprofv3 kernel stats + SQ PMC pass of the shadow kernel on the bench workload (run via gpurun from
# the repo root).   tools/prof_shadow.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-r02}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
KRE=${KREGEX:-frt_jit_shadow}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi "$@" > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit $?
pass() {  # name, counters...
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d "$OUT/$name" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --gi-steps 0 --no-cpu-baseline --no-render-multi > "$OUT/$name.json" 2> "$OUT/$name.err"
}
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pass sq2 SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVES || true
pass fetch FETCH_SIZE || exit $?
pass clk GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
python3 "$R/tools/pmc_summary.py" "$OUT" "$KRE" "${WORKLOAD:-cornell_direct_1920x1080_8x8}" > "$OUT/summary.json" || true
cat "$OUT/summary.json"
ls "$OUT"
