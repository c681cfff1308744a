#!/bin/bash
# PMC passes of the headline shadow kernels (frt_jit_shadow, frt_jit_beam) plus kernel-trace stats,
# run via gpurun from the repo root. Summaries: gpurun_out/prof_TAG/pmc_<kernel>.json
set -o pipefail
TAG=${1:-shadow}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
H="--steps 1 --warmup 0 --gi-steps 0 --no-cpu-baseline --no-render-multi --scene cornell_direct_1920x1080_8x8"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- python3 "$R/bench.py" $H > "$OUT/kt.json" 2> "$OUT/kt.err" || exit $?
pmc() {  # dir kernel-regex counters...
    local d=$1 kre=$2; shift 2
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" $H > "$OUT/$(basename $d).json" 2> "$OUT/$(basename $d).err"
}
for K in frt_jit_shadow frt_jit_beam; do
    mkdir -p "$OUT/$K"
    pmc $K/sq $K SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
    pmc $K/fetch $K FETCH_SIZE || exit $?
    pmc $K/write $K WRITE_SIZE || exit $?
    pmc $K/clk $K GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
done
cd "$R"
for K in frt_jit_shadow frt_jit_beam; do
    cp -r "$OUT/kt" "$OUT/$K/kt"
    python3 tools/pmc_summary.py "$OUT/$K" "$K" cornell_direct_1920x1080_8x8 > "$OUT/pmc_$K.json" || exit $?
    python3 -c "import json; d=json.load(open('$OUT/pmc_$K.json')); print('$K', {k: round(v, 3) if isinstance(v, float) else v for k, v in d.items() if 'per_wave' in k or 'frac' in k or 'rocprof_avg' in k or 'bytes' in k})"
done
