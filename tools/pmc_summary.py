#!/usr/bin/env python3
"""Summarise a profiling directory (tools/prof_shadow.sh): rocprof kernel stats of the kernel and every
PMC pass's counters per launch of it. FETCH_SIZE / WRITE_SIZE (KiB) become bytes per launch; the
MI355X guide's x2 correction for wide streaming reads is not applied (the shadow kernel's loads are
8-byte broadcast loads). The summary carries device_source_sha16, the hash of the device sources
(bench.device_source_sha) the pass ran on.

  python tools/pmc_summary.py gpurun_out/prof_TAG frt_jit_shadow cornell_direct_1920x1080_8x8
"""
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import device_source_sha  # noqa: E402  (bench.py's pairing rule: latest_pmc)

out, kre, workload = sys.argv[1], sys.argv[2], sys.argv[3]
# the kernel's own name, not a longer one it prefixes ("frt_jit_sub" is not "frt_jit_subtile", "k_shade" not
# "k_shade_lit"): the name bounded by characters that cannot continue an identifier
kpat = re.compile(r"(?<![A-Za-z0-9_])(?:%s)(?![A-Za-z0-9_])" % kre)
# the device sources this pass measured (bench.py pairs a summary only with live times of the same sources)
res = {"kernel": sys.argv[4] if len(sys.argv) > 4 else kre, "workload": workload,
       "device_source_sha16": device_source_sha()}
for f in glob.glob(out + "/kt/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if kpat.search(row["Name"]):
            res["rocprof_avg_ms"] = float(row["AverageNs"]) / 1e6
            res["rocprof_calls"] = int(row["Calls"])
            res["rocprof_percentage"] = float(row["Percentage"])
for d in sorted(os.listdir(out)):
    if d == "kt" or not os.path.isdir(os.path.join(out, d)):
        continue
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob("%s/%s/**/*counter_collection.csv" % (out, d), recursive=True):
        for row in csv.DictReader(open(f)):
            if kpat.search(row["Kernel_Name"]):
                tot[row["Counter_Name"]] += float(row["Counter_Value"])
                disp[row["Counter_Name"]].add(row["Dispatch_Id"])
    for k, v in tot.items():
        n = max(1, len(disp[k]))
        if k in ("FETCH_SIZE", "WRITE_SIZE"):
            res[k.lower() + "_bytes_per_launch"] = v * 1024.0 / n
        else:
            res[k + "_per_launch"] = v / n
if "SQ_WAVES_per_launch" in res and "SQ_INSTS_VALU_per_launch" in res:
    res["valu_insts_per_wave"] = res["SQ_INSTS_VALU_per_launch"] / res["SQ_WAVES_per_launch"]
    res["salu_insts_per_wave"] = res.get("SQ_INSTS_SALU_per_launch", 0.0) / res["SQ_WAVES_per_launch"]
if "SQ_WAVE_CYCLES_per_launch" in res:
    wc = res["SQ_WAVE_CYCLES_per_launch"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k + "_per_launch" in res:
            res[k.lower() + "_frac_of_wave_cycles"] = res[k + "_per_launch"] / wc
json.dump(res, sys.stdout, indent=1)
print()
