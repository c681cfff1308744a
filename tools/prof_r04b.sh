#!/bin/bash
# Round-4 profiles of the headline frame after the beam hierarchy (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the headline frames (no GI), the bench's own settings
#   2. PMC passes of each named kernel on the same workload: instruction counts / waits, FETCH, WRITE, clocks, and
#      (k_shade_lit) the binary64 instruction mix for its FP64 roofline
# One counter block set per pass (rocprofv3 does not split passes). Summaries: gpurun_out/prof_TAG/pmc_*.json
#   TAG=r04b KT=1 KERNELS="frt_jit_beam_list frt_jit_sub" bash tools/prof_r04b.sh
set -o pipefail
TAG=${TAG:-r04b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
H="--scene cornell_direct_1920x1080_8x8 --gi-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy"
if [ -n "$KT" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 1 $H > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit $?
fi
pmc() {  # dir kernel-regex counters...
    local d=$1 kre=$2; shift 2
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 $H > "$OUT/$d.json" 2> "$OUT/$d.err"
}
for K in $KERNELS; do
    KRE="(^|::)$K(\(|<|\$)"
    mkdir -p "$OUT/$K"
    pmc $K/sq "$KRE" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
    pmc $K/fetch "$KRE" FETCH_SIZE || exit $?
    pmc $K/write "$KRE" WRITE_SIZE || exit $?
    pmc $K/clk "$KRE" GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
    if [ "$K" = "k_shade_lit" ] || [ "$K" = "k_trace" ]; then
        pmc $K/f64 "$KRE" SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU || exit $?
    fi
done
cd "$R"
for K in $KERNELS; do
    cp -r "$OUT/kt" "$OUT/$K/kt" 2>/dev/null
    python3 tools/pmc_summary.py "$OUT/$K" "(^|::)$K(\(|<|\$)" cornell_direct_1920x1080_8x8 "$K" > "$OUT/pmc_$K.json" || exit $?
done
ls "$OUT"
