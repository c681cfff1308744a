#!/bin/bash
# Round-2 profiles (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the default bench (headline direct frames + one GI frame)
#   2. PMC passes of the per-ray shadow kernel (frt_jit_shadow) and the pair kernel (frt_jit_beam) on the
#      headline workload (cornell_direct_1920x1080_8x8)
#   3. PMC passes of the final-gather estimate (k_gather_est) on cornell_gi_480x270_8x8
# One counter block set per pass (rocprofv3 does not split passes). Summaries: gpurun_out/prof_TAG/*.json
set -o pipefail
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --gi-steps 1 --no-cpu-baseline --no-render-multi > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit $?
pmc() {  # dir kernel-regex bench-args -- counters...
    local d=$1 kre=$2 bargs=$3; shift 3
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --gi-steps 0 --no-cpu-baseline --no-render-multi $bargs > "$OUT/$d.json" 2> "$OUT/$d.err"
}
H="--scene cornell_direct_1920x1080_8x8"
G="--scene cornell_gi_480x270_8x8"
for K in frt_jit_shadow frt_jit_beam; do
    mkdir -p "$OUT/$K"
    pmc $K/sq $K "$H" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
    pmc $K/fetch $K "$H" FETCH_SIZE || exit $?
    pmc $K/write $K "$H" WRITE_SIZE || exit $?
    pmc $K/clk $K "$H" GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
done
K=k_gather_est
mkdir -p "$OUT/$K"
pmc $K/sq $K "$G" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pmc $K/lds $K "$G" SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES || exit $?
pmc $K/fetch $K "$G" FETCH_SIZE || exit $?
pmc $K/write $K "$G" WRITE_SIZE || exit $?
pmc $K/clk $K "$G" GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
cd "$R"
for K in frt_jit_shadow frt_jit_beam; do
    cp -r "$OUT/kt" "$OUT/$K/kt"
    python3 tools/pmc_summary.py "$OUT/$K" "$K" cornell_direct_1920x1080_8x8 > "$OUT/pmc_$K.json" || exit $?
done
mkdir -p "$OUT/k_gather_est/kt"
python3 tools/pmc_summary.py "$OUT/k_gather_est" k_gather_est cornell_gi_480x270_8x8 > "$OUT/pmc_k_gather_est.json" || exit $?
ls "$OUT"
