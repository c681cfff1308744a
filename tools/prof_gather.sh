#!/bin/bash
# k_gather_est profiles on cornell_gi_480x270_8x8 (run via gpurun from the repo root): kernel trace
# stats, then PMC passes (SQ issue/wait, LDS, FETCH_SIZE, WRITE_SIZE, clocks), one block set per pass.
# Summary: gpurun_out/prof_TAG/pmc_k_gather_est.json (tools/pmc_summary.py)
set -o pipefail
TAG=${1:-gather}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
K=k_gather_est
G="--scene cornell_gi_480x270_8x8"
mkdir -p "$OUT/$K"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$K/kt" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --gi-steps 0 --no-cpu-baseline --no-render-multi $G > "$OUT/kt.json" 2> "$OUT/kt.err" || exit $?
pmc() {  # dir counters...
    local d=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -f csv -d "$OUT/$K/$d" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --gi-steps 0 --no-cpu-baseline --no-render-multi $G > "$OUT/$d.json" 2> "$OUT/$d.err"
}
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pmc lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES || exit $?
pmc fetch FETCH_SIZE || exit $?
pmc write WRITE_SIZE || exit $?
pmc clk GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
cd "$R"
python3 tools/pmc_summary.py "$OUT/$K" $K cornell_gi_480x270_8x8 > "$OUT/pmc_$K.json" || exit $?
cat "$OUT/pmc_$K.json"
