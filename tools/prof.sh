#!/bin/bash
# rocprofv3 kernel stats + PMC passes (one counter block set per pass) of a bench workload, summarised
# per kernel with tools/pmc_summary.py (run via gpurun from the repo root).
#   tools/prof.sh TAG SCENE "KERNEL1 KERNEL2 ..." [extra bench args]
set -o pipefail
TAG=$1; SC=$2; KS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="--scene $SC --gi-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy --shipped-steps 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 $B > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit $?
KRE=$(echo $KS | tr ' ' '|')
pmc() {  # dir counters...
    local d=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 $B > "$OUT/$d.json" 2> "$OUT/$d.err"
}
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pmc f64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS || exit $?
pmc fetch FETCH_SIZE || exit $?
pmc write WRITE_SIZE || exit $?
pmc clk GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
cd "$R"
for K in $KS; do
    python3 tools/pmc_summary.py "$OUT" "$K" "$SC" > "$OUT/pmc_$K.json" || exit $?
done
ls "$OUT"
