"""Busy and idle time per frame in a rocprofv3 kernel trace (tools/rank_trace.py): frames split where the GPU idles
more than 150 us (the host's synchronize and timing between frames), then per frame the kernels' union on the timeline
against its span, and the last frame's timeline.   python tools/gaps.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:44]) for r in csv.DictReader(open(sys.argv[1]))))
groups, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if b[0] - a[1] > 150_000:
        groups.append(cur)
        cur = []
    cur.append(b)
groups.append(cur)
for gi, g in enumerate(groups):
    span = g[-1][1] - g[0][0]
    busy, end = 0, g[0][0]
    for s, e, _ in g:
        busy += max(0, e - max(s, end))
        end = max(end, e)
    print("frame %d: %d kernels, span %.3f ms, busy %.3f ms, idle %.3f ms" % (gi, len(g), span / 1e6, busy / 1e6, (span - busy) / 1e6))
g = groups[-1]
end = g[0][0]
print("last frame timeline (gap before, duration, kernel):")
for s, e, name in g:
    print("  %7.1f us  %8.1f us  %s" % ((s - end) / 1e3, (e - s) / 1e3, name))
    end = max(end, e)
