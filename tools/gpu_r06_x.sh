#!/bin/bash
# round 6 (late): the HIP runtime's active wait before a host synchronize sleeps (ROC_ACTIVE_WAIT_TIMEOUT, us): the
# 8-rank share's frame times (tools/rank_trace.py 8) and the headline frame (tools/gpu_ab.sh) at the default and at
# 1000 us
set -o pipefail
mkdir -p gpurun_out
for w in default 1000; do
  if [ $w = default ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$w; fi
  echo "== rank share, ROC_ACTIVE_WAIT_TIMEOUT=$w"
  timeout -k 10 300 python3 tools/rank_trace.py 8 12 > gpurun_out/rankwait_$w.txt 2>&1 || { tail -5 gpurun_out/rankwait_$w.txt; exit 1; }
  grep "^frame" gpurun_out/rankwait_$w.txt | tail -8
done
unset ROC_ACTIVE_WAIT_TIMEOUT
bash tools/gpu_ab.sh cornell_direct_1920x1080_8x8 wait "FRT_NOP=0" "ROC_ACTIVE_WAIT_TIMEOUT=1000" "FRT_NOP=0" "ROC_ACTIVE_WAIT_TIMEOUT=1000" || exit 1
