"""Busy and idle time of the last frame in a rocprofv3 kernel trace (tools/rank_trace.py): the kernels' union on the
timeline against the frame's span, and the largest gaps.   python tools/gaps.py <kernel_trace.csv> [frames]"""
import csv
import sys

rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in csv.DictReader(open(sys.argv[1]))))
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 6
# frames are separated by the host's torch.cuda.synchronize: split at gaps > 1 ms
groups, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if b[0] - a[1] > 1_000_000:
        groups.append(cur)
        cur = []
    cur.append(b)
groups.append(cur)
g = groups[-1]
span = g[-1][1] - g[0][0]
busy, end = 0, g[0][0]
gaps = []
for s, e, name in g:
    if s > end:
        gaps.append((s - end, name))
    busy += max(0, e - max(s, end))
    end = max(end, e)
print("frames %d, last frame: %d kernels, span %.3f ms, busy %.3f ms, idle %.3f ms" % (len(groups), len(g), span / 1e6, busy / 1e6, (span - busy) / 1e6))
for d, name in sorted(gaps, reverse=True)[:25]:
    print("  gap %.1f us before %s" % (d / 1e3, name))
