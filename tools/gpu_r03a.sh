#!/bin/bash
# round-3 GPU check: the -m gpu suite, the box's CPU share, then the non-shadow kernel profiles
set -o pipefail
mkdir -p gpurun_out
{ nproc; python3 -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/pids.max 2>&1; } > gpurun_out/box_cpu.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r03a.log 2>&1 || { tail -40 gpurun_out/pytest_r03a.log; exit 1; }
tail -3 gpurun_out/pytest_r03a.log
bash tools/prof_rest.sh r03
