#!/bin/bash
# The GI frame at full size (cornell_gi_1920x1080_8x8; run via gpurun from the repo root): rocprofv3
# --kernel-trace --stats of one frame and PMC passes over k_gather_est (one counter block set per pass).
# Summary: gpurun_out/gifull_TAG/pmc_k_gather_est.json
set -o pipefail
TAG=${1:-r03}
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
cd "$R"
python3 tools/pmc_summary.py "$OUT" k_gather_est $SC > "$OUT/pmc_k_gather_est.json" || exit $?
ls "$OUT"
