#!/bin/bash
# SQ-level counters for the traversal kernels (debug/profiling aid; run via gpurun from the repo root)
set -o pipefail
TAG=${1:-sq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
    local name=$1; shift
    timeout -k 10 200 rocprofv3 --pmc "$@" --kernel-include-regex "k_shadow|k_trace" -f csv -d "$OUT/$name" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS &&
run b SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQC_DCACHE_HITS SQC_DCACHE_MISSES
