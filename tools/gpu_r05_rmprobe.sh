#!/bin/bash
# round 5: the drop-in's per-process cost (tools/rm_probe.py, fresh processes) and the host round-trip latency
# (tools/microbench/sync.hip, built into variants/sync_bench)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do timeout -k 10 120 python tools/rm_probe.py ${SCENE:-cornell_direct_1920x1080_8x8} > gpurun_out/rm_probe_$i.txt 2>&1 || { tail -5 gpurun_out/rm_probe_$i.txt; exit 1; }; grep JSON gpurun_out/rm_probe_$i.txt | cut -c1-2500; done
timeout -k 10 120 python tools/rm_probe.py ${SCENE:-cornell_direct_1920x1080_8x8} > gpurun_out/rm_probe_4.txt 2>&1 && grep JSON gpurun_out/rm_probe_4.txt | cut -c1-2500
