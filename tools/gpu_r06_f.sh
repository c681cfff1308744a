#!/bin/bash
# round 6: render_multi with 1 / 2 / 4 handles on device 0 (tools/rm_handles_probe.py), then a kernel trace of the
# headline (rocprofv3 --kernel-trace --stats) for the per-kernel picture
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/rm_handles_probe.py cornell_direct_1920x1080_8x8 > gpurun_out/rm_handles.txt 2> gpurun_out/rm_handles.err || { tail -5 gpurun_out/rm_handles.err; exit 1; }
grep JSON gpurun_out/rm_handles.txt
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/kt_r06f" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --gi-steps 0 --shipped-steps 0 --no-cpu-baseline --no-render-multi --no-scaling-proxy \
    > "$R/gpurun_out/kt_r06f.json" 2> "$R/gpurun_out/kt_r06f.err" || exit 1
cd "$R" && ls gpurun_out/kt_r06f
