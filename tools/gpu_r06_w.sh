#!/bin/bash
# round 6 (late): one rank's share of an 8-rank headline frame (tools/rank_trace.py 8), rocprofv3 kernel + memory-copy
# trace, then the busy / idle split per frame and the last frame's timeline (tools/gaps.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rank8
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d "$OUT" -o run -- python3 "$R/tools/rank_trace.py" 8 6 \
    > "$OUT/frames.txt" 2> "$OUT/err.txt" || { tail -5 "$OUT/err.txt"; exit 1; }
cd "$R"
cat "$OUT/frames.txt"
f=$(find "$OUT" -name "*kernel_trace.csv" | head -1)
python3 tools/gaps.py "$f" > gpurun_out/rank8_gaps.txt
m=$(find "$OUT" -name "*memory_copy_trace.csv" | head -1)
[ -n "$m" ] && cp "$m" gpurun_out/rank8_copies.csv
head -8 gpurun_out/rank8_gaps.txt
