#!/bin/bash
# round 5: k_gather_est's SQ counters on one GI frame (default order): SC=<scene> tools/pmc_gi.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gi
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SC=${SC:-cornell_gi_480x270_8x8}
pass() {
  local d=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex k_gather_est -f csv -d "$OUT/$d" -o run -- \
      python3 "$R/tools/gi_frame.py" $SC > "$OUT/$d.txt" 2>&1
}
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INST_CYCLES_VMEM || exit $?
pass sq3 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F64 || exit $?
pass clk GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
cd "$R" && for d in "$OUT"/*/; do echo "== $d"; python3 tools/pmc_sum.py "$d"; done > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
