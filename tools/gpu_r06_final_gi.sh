#!/bin/bash
# round 6 final evidence (GI): rocprofv3 kernel stats of one full-size GI frame and PMC passes over k_gather_est
# (tools/prof_gi_full.sh without its instrumented-build step; the phase split is profiles/r06_gi_est_phases.txt)
set -o pipefail
TAG=${1:-r06z}
SC=cornell_gi_1920x1080_8x8
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gifull_$TAG
mkdir -p "$OUT"
B="--scene $SC --gi-steps 0 --no-cpu-baseline --no-render-multi --steps 1 --warmup 0"
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
