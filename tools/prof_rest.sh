#!/bin/bash
# PMC passes over the headline frame's kernels outside the shadow pass (k_shade, k_prepare, k_trace,
# k_combine, k_resolve) plus the headline-only kernel-trace stats (run via gpurun from the repo root).
#   tools/prof_rest.sh TAG [scene]
# One counter block set per pass (rocprofv3 does not split passes). Summaries: gpurun_out/rest_TAG/pmc_*.json
set -o pipefail
TAG=${1:-r03}
SC=${2:-cornell_direct_1920x1080_8x8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rest_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="--scene $SC --gi-steps 0 --no-cpu-baseline --no-render-multi"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 $B > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit $?
KRE='k_shade|k_prepare|k_trace|k_combine|k_resolve'
pmc() {  # dir counters...
    local d=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 $B > "$OUT/$d.json" 2> "$OUT/$d.err"
}
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pmc mem SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_FLAT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU || exit $?
pmc fetch FETCH_SIZE || exit $?
pmc write WRITE_SIZE || exit $?
pmc clk GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
cd "$R"
for K in k_shade k_prepare k_trace k_combine k_resolve; do
    python3 tools/pmc_summary.py "$OUT" "$K" "$SC" > "$OUT/pmc_$K.json" || exit $?
done
ls "$OUT"
