#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (the last line of the file given)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
print("headline ms %.3f  value %.0f  ref-equiv %.0f" % (d["ms_per_step"], d["value"], d.get("reference_equivalent_mrays_s") or 0))
print("  kernels", {k: round(v, 2) for k, v in d["kernel_ms_per_frame"].items()})
print("  sub", {k: round(v, 2) for k, v in d["sub_ms_per_frame"].items()})
r = d.get("roofline", {})
print("  roofline", r.get("kernel"), r.get("bound"), r.get("frac"), r.get("pmc_rejected", ""))
if d.get("shipped"):
    s = d["shipped"]
    print("shipped ms %.3f" % s["ms_per_step"], {k: round(v, 2) for k, v in s["kernel_ms_per_frame"].items()})
    print("  sub", {k: round(v, 2) for k, v in s["sub_ms_per_frame"].items()})
if d.get("gi"):
    g = d["gi"]
    print("gi ms %.1f" % g["ms_per_step"], {k: round(v, 1) for k, v in g["kernel_ms_per_frame"].items()},
          g.get("gather_est"))
print("render_multi", {k: v for k, v in d.items() if k.startswith("render_multi_wall")})
if d.get("render_multi_phases_warm"):
    print("  warm phases", {k: round(v, 1) for k, v in d["render_multi_phases_warm"].items() if v})
if d.get("scaling_proxy"):
    for k, v in d["scaling_proxy"].items():
        if isinstance(v, dict):
            print("proxy", k, {n: e.get("predicted_efficiency") for n, e in v.items()})
if d.get("cpu_baseline"):
    print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
