#!/bin/bash
# Round-4 profiles of the headline frame (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the headline direct frames (no GI)
#   2. PMC passes (instruction counts / waits, FETCH, WRITE, clocks) of the shadow pass's three kernels
#      (frt_jit_tile, frt_jit_beam_list, frt_jit_shadow) on the same workload
# One counter block set per pass (rocprofv3 does not split passes). Summaries: gpurun_out/prof_TAG/pmc_*.json
set -o pipefail
TAG=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
H="--scene cornell_direct_1920x1080_8x8 --gi-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 $H > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit $?
pmc() {  # dir kernel-regex counters...
    local d=$1 kre=$2; shift 2
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 $H > "$OUT/$d.json" 2> "$OUT/$d.err"
}
for K in ${KERNELS:-frt_jit_shadow frt_jit_beam_list frt_jit_tile}; do
    mkdir -p "$OUT/$K"
    pmc $K/sq $K SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
    pmc $K/fetch $K FETCH_SIZE || exit $?
    pmc $K/write $K WRITE_SIZE || exit $?
    pmc $K/clk $K GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
done
cd "$R"
for K in ${KERNELS:-frt_jit_shadow frt_jit_beam_list frt_jit_tile}; do
    cp -r "$OUT/kt" "$OUT/$K/kt"
    python3 tools/pmc_summary.py "$OUT/$K" "$K" cornell_direct_1920x1080_8x8 > "$OUT/pmc_$K.json" || exit $?
done
ls "$OUT"
