#!/bin/bash
# VALU / SALU instruction counts of k_shadow under several FRT_WALK_FLAGS (profiling aid; via gpurun)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_ab
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for f in "$@"; do
  FRT_WALK_FLAGS=$f timeout -k 10 200 rocprofv3 --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64} \
    --kernel-include-regex "k_shadow" -f csv -d "$OUT/f$f" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> "$OUT/f$f.err" || exit 1
done
