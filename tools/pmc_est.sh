#!/bin/bash
# PMC passes over k_gather_est on a GI scene (run via gpurun from the repo root); counters list first.
#   tools/pmc_est.sh TAG [scene]
set -o pipefail
TAG=${1:-est}; SC=${2:-cornell_gi_480x270_8x8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcest_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
B="--scene $SC --gi-steps 0 --no-cpu-baseline --no-render-multi --steps 1 --warmup 0"
pmc() {  # dir counters...
    local d=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex k_gather_est -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" $B > "$OUT/$d.json" 2> "$OUT/$d.err"
}
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pmc act SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS || exit $?
pmc tcc TCC_HIT_sum TCC_MISS_sum || exit $?
pmc tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit $?
pmc fetch FETCH_SIZE || exit $?
cd "$R"
python3 tools/pmc_summary.py "$OUT" k_gather_est "$SC" > "$OUT/pmc_k_gather_est.json"
cat "$OUT/pmc_k_gather_est.json"
