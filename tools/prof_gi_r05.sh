#!/bin/bash
# round 5: the GI frame at full size (cornell_gi_1920x1080_8x8): rocprofv3 --kernel-trace --stats of one frame, then
# PMC passes over k_gather_est (one counter block set per pass), summarised by tools/pmc_summary.py
set -o pipefail
TAG=${1:-r05}
SC=cornell_gi_1920x1080_8x8
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gifull_$TAG
mkdir -p "$OUT"
B="--scene $SC --gi-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy --shipped-steps 0 --steps 1 --warmup 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- python3 "$R/bench.py" $B > "$OUT/kt.json" 2> "$OUT/kt.err" || exit $?
pmc() {
    local d=$1; shift
    timeout -s KILL 400 rocprofv3 --pmc "$@" --kernel-include-regex k_gather_est -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" $B > "$OUT/$d.json" 2> "$OUT/$d.err"
}
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pmc fetch FETCH_SIZE || exit $?
pmc write WRITE_SIZE || exit $?
pmc tcc TCC_HIT_sum TCC_MISS_sum || exit $?
pmc clk GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
cd "$R"
python3 tools/pmc_summary.py "$OUT" k_gather_est "$SC" > "$OUT/pmc_k_gather_est.json" || exit $?
cat "$OUT/pmc_k_gather_est.json"
