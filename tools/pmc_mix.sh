#!/bin/bash
# Instruction-mix PMC passes (VALU classes, SALU, LDS, I-cache) over the kernels matching a regex on one
# scene (run via gpurun from the repo root).   tools/pmc_mix.sh TAG KERNEL_REGEX SCENE
set -o pipefail
TAG=$1; KRE=$2; SC=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/mix_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="--scene $SC --gi-steps 0 --no-cpu-baseline --no-render-multi --steps 1 --warmup 0"
pmc() {
    local d=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" $B > "$OUT/$d.json" 2> "$OUT/$d.err"
}
pmc p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 || exit $?
pmc p2 SQ_WAVES SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS || exit $?
pmc p3 SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VMEM_RD || exit $?
pmc p4 SQC_ICACHE_MISSES SQC_ICACHE_HITS || exit $?
pmc p5 GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
cd "$R"
for K in $(echo "$KRE" | tr '|' ' '); do
    python3 tools/pmc_summary.py "$OUT" "$K" "$SC" > "$OUT/pmc_$K.json" || exit $?
done
ls "$OUT"
