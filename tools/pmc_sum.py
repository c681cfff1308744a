#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter CSVs per kernel (tools/pmc_shadow.sh output dir)."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(glob.glob(out + "/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0]
        tot[(k, row["Counter_Name"])] += float(row["Counter_Value"])
        disp[k].add((f, row["Dispatch_Id"]))
for (k, c), v in sorted(tot.items()):
    print("%-40s %-28s %16.0f  (%d dispatches)" % (k[:40], c, v, len(disp[k])))
