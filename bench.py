#!/usr/bin/env python3
"""bench.py — frt-mi355x headline benchmark.

Workload (BASELINE.json north_star target / configs[4] camera): cornell_box at
1920x1080 with an 8x8 CMJ sub-pixel grid (64 spp), full reflection/refraction
recursion (path length 5), one 10x10 area light; GI off and a single-row light
cache — the deterministic parity variant the tests check against the oracle
(tests/test_gpu_parity.py) and, at 1/64 of the pixels, against the reference
itself (golden cornell_direct_240x135_8x8). The scene is the reference
codegen's own main.c (tests/golden/scenes/), built through the drop-in API in
capture mode.

One step = one full frame: every rank renders its interleaved rows on its GPU
(HBM-resident output), then the canvas is gathered on rank 0 over RCCL.
Metric: Mrays/s of rays actually traced (primary + secondary + shadow), summed
over ranks, plus wall-clock per frame; reference-equivalent Mrays/s (the rays the
reference would cast, counted by the oracle: zero-weight secondary subtrees
included) are reported beside it. `value` counts every shadow ray, also the ones
the beam stages decide for a whole beam at once; `walked_mrays_s` counts only the
rays walked one by one, and ms_per_step / reference_equivalent_mrays_s are the
figures to compare with the reference.

Also on the same JSON line:
  shipped          the shipped direct-lighting configuration (cornell_box.yml's 65 535-row jittered light cache, GI
                   off) at 1920x1080x64: --shipped-steps frames
  gi               the shipped GI configuration (BASELINE configs[4]: 1M photons per map,
                   8x8 final gather, k = 200) at 1920x1080x64: --gi-steps frames, each with a
                   new seed so photon tracing + map build run inside the timed region
  render_multi_*   wall time of the drop-in entry point itself (flatten, upload, hiprtc
                   compile of the scene kernel, render, copy to the host canvas)
  roofline         the frame's dominant kernel by live HIP-event time (k_shade_lit on the headline) against the
                   peak of the bound its committed PMC pass shows (binary64 FLOPs against the 78.6 TFLOP/s vector
                   peak, instruction issue, or HBM bytes against 8 TB/s); a PMC pass is used only when it was
                   measured on this tree's device sources and its rocprof launch time lies within 20 % of the live
                   one (latest_pmc), otherwise the fields are null and pmc_rejected says why
  cpu_baseline     the reference's own pthread render_multi on this host's cores, on a
                   bounded sample of the same workload (the same camera at 240x135)

  python bench.py [--gpus N] [--steps K] [--warmup W] [--gi-steps G] [--scene NAME] [--no-cpu-baseline]
  torchrun --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no torchrun environment, bench.py starts torchrun itself
(one rank per GPU) before touching the GPU and exits with its status; a
WORLD_SIZE that disagrees with --gpus is an error (never a silent 1-GPU run).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
ASSETS = os.path.join(GOLDEN, "assets")
DEFAULT_SCENE = "cornell_direct_1920x1080_8x8"
GI_SCENE = "cornell_gi_1920x1080_8x8"
SHIPPED_SCENE = "cornell_shipped_1920x1080_8x8"
CPU_SAMPLE_SCENE = "cornell_direct_240x135_8x8"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD per 2 cycles (SIMD32; binary64
# and transcendental instructions take 2-4x: profiles/r01_microbench_valu.txt) at the 2.4 GHz peak clock
VALU_PEAK_GINST_S = 1024 * 2.4 / 2.0
# SALU issue peak: one scalar unit per CU, one instruction per cycle, shared by the CU's 4 SIMDs
SALU_PEAK_GINST_S = 256 * 2.4
# binary64 vector peak (MI355X spec, 78.6 TFLOP/s): 1024 SIMDs x 16 lanes per cycle x 2 flops (FMA) at 2.4 GHz
# (profiles/r01_microbench_valu.txt measures ~5 SIMD-cycles per wave64 f64 FMA against the 4 of this figure)
FP64_PEAK_TFLOPS = 78.6

# algorithmic HBM bytes of the shadow kernel ("byte model"), reported by the engine per frame
# as stats.shadow_kernel_bytes: per shaded path node the 64-byte ShadowHead it reads (over_point, key,
# material; one cache line) and one 4-byte unshadowed count per light it writes. Light points and
# sample tables (a few KB) stay in cache and are not counted.


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks_if_needed(args) -> None:
    """--gpus N without a torchrun environment: run N ranks under torchrun (a child process,
    started before this process touches the GPU) and exit with its status."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
                   "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), os.path.abspath(__file__)] + sys.argv[1:]
            log("bench: starting %d ranks: %s" % (args.gpus, " ".join(cmd)))
            sys.exit(subprocess.call(cmd))
        return
    if int(env_world) != args.gpus:
        log("bench: --gpus %d but WORLD_SIZE=%s: refusing to measure a different GPU count" % (args.gpus, env_world))
        sys.exit(2)


def reference_rays(name: str):
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f).get(name, {}).get("reference_rays", {}).get("total")


def cpu_baseline(all_threads: bool = False) -> dict | None:
    """The reference's own pthread render_multi on this host, on a bounded sample of the workload:
    the same camera and scene at 240x135 (1/64 of the pixels, 8x8 CMJ), timed with the pool at the CPU quota of
    this process (runtime.cpu_share); with all_threads (--cpu-all-threads) also at os.cpu_count() (the
    reference's own default of one thread per visible CPU: 256 on the GPU box, time-sliced on its 16-CPU
    quota, measured 4.6x slower in round 3), the faster run being the baseline.
    The binary is oracle/_ref/bin/<sample>: built from the reference's sources by oracle/build_ref.sh
    in the build container (a git-ignored artefact that travels with the working tree; no reference
    source is in the repo). Without it, the repository's own C restatement (oracle/, "port") is timed."""
    from fast_ray_tracer_amd.runtime import cpu_share
    rays = reference_rays(CPU_SAMPLE_SCENE)
    exe = os.path.join(ROOT, "oracle", "_ref", "bin", CPU_SAMPLE_SCENE)
    host_cpus = os.cpu_count()
    # the reference's pool sized to the CPUs this process may use: the cgroup quota of the GPU box (16 per
    # GPU) while os.cpu_count() reports the whole machine (256); more threads than the quota only time-slice
    threads = cpu_share()
    if os.path.exists(exe) and rays:
        def run_ref(nt: int):
            stats = "/tmp/frt_bench_ref_stats_%d_%d.json" % (os.getpid(), nt)
            os.makedirs("/tmp/frt_golden/out", exist_ok=True)
            t0 = time.time()
            proc = subprocess.run([exe], cwd=ASSETS, env=dict(os.environ, FRT_REF_STATS=stats, FRT_REF_THREADS=str(nt)),
                                  stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, timeout=600)
            if proc.returncode != 0:
                log("cpu_baseline: reference run failed:", proc.stderr[-500:])
                return None
            st = json.load(open(stats))
            st["wall_seconds"] = time.time() - t0
            return st
        # the pool at this process's CPU quota and at every CPU the machine shows (the reference's own
        # thread-count knob, config.py: threads = CPU count); the faster one is the baseline
        runs = []
        for nt in sorted({threads, host_cpus or threads} if all_threads else {threads}):
            st = run_ref(nt)
            if st is None:
                return None
            runs.append(st)
        best = min(runs, key=lambda r: r["render_multi_seconds"])
        secs = best["render_multi_seconds"]
        return {"value": round(rays / secs / 1e6, 4), "unit": "Mrays/s", "cores": int(best["threads"]),
                "kind": "reference", "threads": int(best["threads"]), "cpu_quota": cpu_share(),
                "host_cpus_visible": host_cpus, "seconds": round(secs, 3),
                "wall_seconds": round(best["wall_seconds"], 3),
                "runs": [{"threads": int(r["threads"]), "value": round(rays / r["render_multi_seconds"] / 1e6, 4),
                          "seconds": round(r["render_multi_seconds"], 3)} for r in runs],
                "sample": "%s: the reference's render_multi (pthread pool) built from /root/reference sources by "
                          "oracle/build_ref.sh, %dx%dx%d spp (the benchmark camera at 1/64 of the pixels), %d "
                          "reference rays counted by the oracle; timed with %s threads (this process's CPU quota%s), "
                          "the faster reported"
                          % (CPU_SAMPLE_SCENE, best["width"], best["height"], best["usteps"] * best["vsteps"], rays,
                             " and ".join(str(int(r["threads"])) for r in runs),
                             " and the %d CPUs the machine shows" % host_cpus if all_threads else "")}
    # checker leg only (never the GPU path): the oracle restatement on the same sample
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    from conftest import load_scene
    scene = load_scene(CPU_SAMPLE_SCENE)
    t0 = time.time()
    _, st = oracle.render(scene, threads=threads, stats=True)
    secs = time.time() - t0
    total = int(st["primary_rays"] + st["secondary_rays"] + st["shadow_rays"])
    return {"value": round(total / secs / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "threads": threads, "cpu_quota": cpu_share(), "host_cpus_visible": host_cpus, "seconds": round(secs, 3),
            "sample": "%s: oracle/ C restatement of the reference (reference build absent), %d threads, %d rays"
                      % (CPU_SAMPLE_SCENE, threads, total)}


PROFILES = os.path.join(ROOT, "profiles")
# the device library's sources: a PMC summary is evidence for the kernels these files compiled to, so
# tools/pmc_summary.py stamps it with their hash and a summary of other sources is not paired with a live time
DEVICE_SOURCES = [os.path.join(ROOT, "include", "frt_device.h")] + [
    os.path.join(ROOT, "fast_ray_tracer_amd", "csrc", f) for f in
    ("frt_camera.hpp", "frt_cols.hpp", "frt_engine.hip", "frt_gi.hpp", "frt_jit.h", "frt_jit.hip", "frt_jit_rt.hpp",
     "frt_math.hpp", "frt_shade.hpp", "frt_shadow.hpp", "frt_traverse.hpp")]
# a PMC pass's rocprof launch time may differ from the live HIP-event time by this much (relative) and still be
# paired with it: more means another build, another workload or another box state, and its rates would be fiction
PMC_TIME_TOL = 0.20


def device_source_sha(paths=None) -> str:
    """sha256 (first 16 hex digits) over the device sources' names and bytes."""
    import hashlib
    h = hashlib.sha256()
    for p in sorted(paths or DEVICE_SOURCES):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def latest_pmc(kernel: str, workload: str, live_avg_ms: float | None = None, profiles_dir: str | None = None):
    """The newest committed PMC summary (profiles/rNN_pmc_*.json) of this kernel on this workload that may be
    paired with a live launch time: it must carry the hash of the device sources it was measured on
    (device_source_sha16, written by tools/pmc_summary.py) equal to this tree's, and its rocprof average launch
    time must lie within PMC_TIME_TOL of live_avg_ms. Returns (path, summary, None), or (None, None, reason)
    when no summary qualifies (reason: why the newest candidate was rejected)."""
    cands = []
    for p in sorted(glob.glob(os.path.join(profiles_dir or PROFILES, "r*_pmc_*.json"))):
        try:
            t = json.load(open(p))
        except (OSError, ValueError):
            continue
        # (older summaries name the kernel by the regex their pass used, "k_shadow<")
        if t.get("kernel", "").rstrip("<") == kernel and t.get("workload") == workload:
            cands.append((p, t))
    if not cands:
        return None, None, "no PMC summary of %s on %s under profiles/" % (kernel, workload)
    sha = device_source_sha()
    reasons = []
    for p, t in reversed(cands):
        name = os.path.basename(p)
        if t.get("device_source_sha16") != sha:
            reasons.append("%s: measured on other device sources (%s, this tree %s)"
                           % (name, t.get("device_source_sha16", "no source hash"), sha))
            continue
        ra = t.get("rocprof_avg_ms")
        if live_avg_ms is not None:
            if not ra or not live_avg_ms or abs(ra - live_avg_ms) > PMC_TIME_TOL * live_avg_ms:
                reasons.append("%s: rocprof launch %s ms vs live %.4f ms (more than %d %% apart)"
                               % (name, ("%.4f" % ra) if ra else "n/a", live_avg_ms or 0.0, round(100 * PMC_TIME_TOL)))
                continue
        return p, t, None
    return None, None, reasons[0]


def issue_block(t: dict, avg_ms: float, units_per_launch: float, unit_name: str) -> dict:
    """VALU and SALU issue rates of one kernel from its committed PMC pass (instructions per launch) over
    the live event-timed launch duration, against the chip's issue peaks."""
    out = {}
    for key, peak, name in (("SQ_INSTS_VALU_per_launch", VALU_PEAK_GINST_S, "valu"),
                            ("SQ_INSTS_SALU_per_launch", SALU_PEAK_GINST_S, "salu")):
        if key in t:
            ginst = t[key] / (avg_ms * 1e-3) / 1e9
            out[name] = {"achieved": round(ginst, 1), "peak": round(peak, 1), "unit": "G wave64 inst/s",
                         "frac": round(ginst / peak, 3),
                         "inst_per_64_" + unit_name: round(64.0 * t[key] / units_per_launch, 1) if units_per_launch else None}
    for k in ("sq_wait_any_frac_of_wave_cycles", "sq_wait_inst_any_frac_of_wave_cycles",
              "sq_active_inst_any_frac_of_wave_cycles"):
        if k in t:
            out[k] = round(t[k], 3)
    return out


def shadow_roofline(d: dict, kernel_ms: dict, launches: dict, workload: str) -> dict:
    """The per-ray shadow kernel (frt_jit_shadow; the generic k_shadow when the scene is not eligible),
    timed by HIP events around its own launches (frt_frame_stats.sub_ms). Algorithmic bytes (engine-side
    shadow_kernel_bytes): per list entry its 8 bytes, per node of an entry its 40-byte ShadowHead once (not per ray:
    the node's rays share it; and at most once per node and launch: the entries of one tile re-read their nodes'
    records from L2) and one 4-byte count, per ray of a multi-row light its 24-byte point.

    bound: "valu-issue" — the kernel moves few bytes (achieved / peak / frac below are its algorithmic
    HBM bytes against the 8 TB/s peak, as the bench contract asks) and is limited by instruction issue on
    both pipes; `issue` holds the VALU and SALU rates from the committed PMC pass of the same kernel on
    the same workload over the live launch time (and the same for the pair kernel, frt_jit_beam)."""
    if d.get("shadow_jit") and d.get("sub_launches", {}).get("frt_jit_shadow"):
        kname = "frt_jit_shadow"
        avg_ms = d["sub_ms"]["frt_jit_shadow"] / d["sub_launches"]["frt_jit_shadow"]
        nl = d["sub_launches"]["frt_jit_shadow"]
    else:
        kname = "k_shadow"
        avg_ms = kernel_ms["shadow"] / max(1, launches["shadow"])
        nl = max(1, launches["shadow"])
    per_launch = d["shadow_kernel_bytes"] / nl
    achieved = per_launch / (avg_ms * 1e-3) / 1e9
    roof = {"bound": "valu-issue" if kname == "frt_jit_shadow" else "hbm", "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "kernel": kname,
            "avg_launch_ms": round(avg_ms, 4), "launches_per_frame": nl,
            "algorithmic_bytes_per_launch": round(per_launch),
            "timing": "HIP events around each launch on the engine stream (frt_frame_stats.sub_ms)"}
    path, t, why = latest_pmc(kname, workload, avg_ms)
    if why:
        roof["pmc_rejected"] = why
    if path:
        if "traffic_bytes_per_launch" in t:
            roof["traffic"] = round(t["traffic_bytes_per_launch"])
        else:  # FETCH_SIZE + WRITE_SIZE (tools/pmc_summary.py, KiB units already converted)
            roof["traffic"] = round(t.get("fetch_size_bytes_per_launch", 0.0) + t.get("write_size_bytes_per_launch", 0.0))
        roof["traffic_source"] = os.path.relpath(path, ROOT)
        if "rocprof_avg_ms" in t:
            roof["rocprof_avg_launch_ms"] = round(t["rocprof_avg_ms"], 4)
        rays_per_launch = (d.get("shadow_rays_walked") or 0) / nl
        roof["issue"] = {kname: issue_block(t, avg_ms, rays_per_launch, "rays")}
        roof["issue"][kname]["source"] = os.path.relpath(path, ROOT)
    # the pair kernels: the node pairs (frt_jit_beam_list after the tile kernel, frt_jit_beam without it; one
    # timer slot) and the tile pairs (frt_jit_tile)
    nb = d.get("sub_launches", {}).get("frt_jit_beam")
    tiled = bool(d.get("shadow_tile_pairs"))
    bname = "frt_jit_beam_list" if tiled else "frt_jit_beam"
    if nb:
        bavg = d["sub_ms"]["frt_jit_beam"] / nb
        fp, ft, why = latest_pmc(bname, workload, bavg)
        pairs_per_launch = (d.get("shadow_pairs") or 0) / nb
        roof.setdefault("issue", {})[bname] = (
            dict(issue_block(ft, bavg, pairs_per_launch, "pairs"), avg_launch_ms=round(bavg, 4),
                 source=os.path.relpath(fp, ROOT)) if fp else {"avg_launch_ms": round(bavg, 4), "pmc_rejected": why})
    for kn, units, uname in (("frt_jit_tile", d.get("shadow_tile_pairs"), "tile_pairs"),
                             ("frt_jit_sub", d.get("shadow_sub_pairs"), "tile_sub_pairs"),
                             ("frt_jit_subtile", d.get("shadow_subtile_pairs"), "subtile_pairs")):
        nt = d.get("sub_launches", {}).get(kn)
        if nt:
            tavg = d["sub_ms"][kn] / nt
            fp, ft, why = latest_pmc(kn, workload, tavg)
            roof.setdefault("issue", {})[kn] = (
                dict(issue_block(ft, tavg, (units or 0) / nt, uname), avg_launch_ms=round(tavg, 4),
                     source=os.path.relpath(fp, ROOT)) if fp else {"avg_launch_ms": round(tavg, 4), "pmc_rejected": why})
    return roof


def frame_roofline(d: dict, kernel_ms: dict, launches: dict, workload: str) -> dict:
    """The frame's dominant kernel by live time (HIP events around its launches in the stats frame: the engine's
    sub-timers for the scene-specialised shadow kernels and k_shade_lit, its per-slot timers for k_trace (level
    0), k_prepare and k_combine_resolve), with the bound its committed PMC pass on the same workload shows:
      * "valu-fp64" (k_shade_lit, k_trace): achieved = the pass's binary64 FLOPs per launch (64 x (ADD + MUL +
        TRANS) + 128 x FMA wave-instructions) over the live launch time, against the 78.6 TFLOP/s binary64
        vector peak; `issue` adds the VALU / SALU issue rates;
      * "valu-issue" (the pair and per-ray shadow kernels): the issue rates as `roofline_shadow_pass` gives them;
      * "hbm" otherwise: FETCH_SIZE + WRITE_SIZE per launch over the live launch time against 8 TB/s.
    `traffic` is FETCH_SIZE + WRITE_SIZE per launch of the same PMC run in every case."""
    subs, sl = d.get("sub_ms", {}), d.get("sub_launches", {})
    cands = {}
    for k in ("k_shade_lit", "frt_jit_beam", "frt_jit_shadow", "frt_jit_tile", "frt_jit_sub", "frt_jit_subtile"):
        if sl.get(k):
            cands[k] = (subs[k], sl[k])
    slots = [("k_trace", "trace_primary"), ("k_prepare", "prepare"), ("k_combine_resolve", "resolve")]
    if not d.get("shadow_jit"):
        slots.append(("k_shadow", "shadow"))  # (the generic walk: scenes the generator does not take)
    for k, slot in slots:
        if launches.get(slot):
            cands[k] = (kernel_ms[slot], launches[slot])
    if not cands:
        return {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None}
    dom = max(cands, key=lambda k: cands[k][0])
    ms, nl = cands[dom]
    pname = "frt_jit_beam_list" if dom == "frt_jit_beam" and d.get("shadow_tile_pairs") else dom
    avg = ms / nl
    roof = {"kernel": pname, "avg_launch_ms": round(avg, 4), "launches_per_frame": nl, "ms_per_frame": round(ms, 3),
            "timing": "HIP events around each launch on the engine stream (frt_frame_stats)",
            "candidates_ms_per_frame": {k: round(v[0], 3) for k, v in sorted(cands.items(), key=lambda kv: -kv[1][0])}}
    path, t, why = latest_pmc(pname, workload, avg)
    found = path is not None
    t = t or {}
    traffic = (t.get("fetch_size_bytes_per_launch", 0.0) + t.get("write_size_bytes_per_launch", 0.0)) if found else None
    f64 = [t.get("SQ_INSTS_VALU_%s_F64_per_launch" % x) for x in ("ADD", "MUL", "FMA", "TRANS")]
    if not found:
        # no counter evidence that matches this build and this launch time: nothing to divide, say why
        roof.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "pmc_rejected": why})
    elif all(v is not None for v in f64):
        flops = 64.0 * (f64[0] + f64[1] + f64[3]) + 128.0 * f64[2]
        ach = flops / (avg * 1e-3) / 1e12
        roof.update({"bound": "valu-fp64", "achieved": round(ach, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(ach / FP64_PEAK_TFLOPS, 4), "fp64_flops_per_launch": round(flops),
                     "fp64_flops_note": "64 x the wave instruction counts of the PMC pass (128 x for FMA): lanes a wave "
                                        "masks off are counted as working, so the true FLOP rate is at most this"})
    elif pname.startswith("frt_jit"):
        roof.update({"bound": "valu-issue", "achieved": None, "peak": None, "unit": None, "frac": None,
                     "note": "instruction-issue bound; see roofline_shadow_pass.issue for the VALU / SALU fractions"})
    else:
        ach = traffic / (avg * 1e-3) / 1e9 if traffic else None
        roof.update({"bound": "hbm", "achieved": round(ach, 1) if ach else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None})
    roof["traffic"] = round(traffic) if traffic else None
    if found:
        roof["source"] = os.path.relpath(path, ROOT)
        roof["issue"] = issue_block(t, avg, 1.0, "launch")
        if "rocprof_avg_ms" in t:
            roof["rocprof_avg_launch_ms"] = round(t["rocprof_avg_ms"], 4)
    return roof


def gather_roofline(gd: dict) -> dict:
    """k_gather_est (the GI frame's dominant kernel): the photon-map estimate per final-gather ray.
    Algorithmic bytes per query (profiles/r03_gi_estimate_counters.json: device counters of the estimate,
    tools/prof_gi_full.sh; the algorithm has not changed since): the binary32 positions of the candidates it
    scans (16 B each), the 80-byte records of the photons it uses, its 96-byte request and 24-byte result.
    `achieved` = that per query x this frame's queries per launch over the live event-timed launch duration;
    `traffic` = the PMC FETCH_SIZE (x2, the guide's gfx950 correction for wide coalesced reads) + WRITE_SIZE per
    launch of the same workload (the newest profiles/r*_pmc_k_gather_est_cornell_gi_1920x1080_8x8.json).

    bound: "valu-issue" since round 5. The requests are estimated in the Morton order of their points, dealt to
    per-XCD queues, so one XCD's queries share the photons in its L2 (TCC hit rate 37 % -> 96 %, FETCH_SIZE / 21,
    profiles/r05_ab_gi_sort.txt): the ~20 KB a query reads are L2 hits, the byte rate below is an L2-request
    rate (not HBM), and `issue` holds the VALU / SALU issue rates of the PMC pass over the live launch time."""
    n = gd["sub_launches"]["k_gather_est"]
    avg_ms = gd["sub_ms"]["k_gather_est"] / n
    roof = {"bound": "valu-issue", "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
            "kernel": "k_gather_est", "avg_launch_ms": round(avg_ms, 4), "launches_per_frame": n,
            "bytes_model": "l2_request_gbs: the byte model counts every byte the estimate requests from the memory "
                           "system (candidate positions, photon records, request, result) over the live launch time; "
                           "with the requests in spatial order they hit the XCDs' L2, so it is not an HBM rate "
                           "(traffic is the HBM side). achieved / peak / frac: the VALU issue rate"}
    model = os.path.join(ROOT, "profiles", "r03_gi_estimate_counters.json")
    if os.path.exists(model):
        m = json.load(open(model))
        per_query = m["algorithmic_bytes_per_query"]
        per_launch = per_query * gd["gather_rays"] / n
        ach = per_launch / (avg_ms * 1e-3) / 1e9
        roof.update({"l2_request_gbs": round(ach, 1),
                     "algorithmic_bytes_per_query": round(per_query, 1),
                     "algorithmic_bytes_per_launch": round(per_launch),
                     "candidates_per_query": round(m["candidates_read_per_query"], 1),
                     "records_per_query": round(m["records_read_per_query"], 1),
                     "model_source": os.path.relpath(model, ROOT)})
    path, t, why = latest_pmc("k_gather_est", GI_SCENE, avg_ms)
    if why:
        roof["pmc_rejected"] = why
    if path:
        traffic = 2.0 * t.get("fetch_size_bytes_per_launch", 0.0) + t.get("write_size_bytes_per_launch", 0.0)
        queries = gd["gather_rays"] / n
        roof.update({"traffic": round(traffic), "traffic_source": os.path.relpath(path, ROOT),
                     "rocprof_avg_launch_ms": round(t.get("rocprof_avg_ms", 0.0), 4),
                     # per query: the launch's counts over its queries (the estimate's waves take requests
                     # from a queue, so waves and queries are not in a fixed ratio)
                     "valu_insts_per_query": round(t["SQ_INSTS_VALU_per_launch"] / queries, 1),
                     "salu_insts_per_query": round(t["SQ_INSTS_SALU_per_launch"] / queries, 1),
                     "wait_any_frac": round(t.get("sq_wait_any_frac_of_wave_cycles", 0.0), 3),
                     "issue": issue_block(t, avg_ms, queries, "queries")})
        v = roof["issue"].get("valu")
        if v:  # achieved / peak / frac: the VALU issue rate of the PMC pass over the live launch time
            roof.update({"achieved": v["achieved"], "peak": v["peak"], "unit": v["unit"], "frac": v["frac"]})
        if "TCC_HIT_sum_per_launch" in t and "TCC_MISS_sum_per_launch" in t:
            hm = t["TCC_HIT_sum_per_launch"] + t["TCC_MISS_sum_per_launch"]
            roof["l2_hit_rate"] = round(t["TCC_HIT_sum_per_launch"] / hm, 4) if hm else None
    return roof


def scaling_proxy(renderer, shard, height: int, frame_ms_1: float, ns=(2, 4, 8), reps: int = 2, seed_of=None,
                  batch_samples: int = 0) -> dict:
    """The multi-GPU split measured on this one GPU: for N ranks, rank r renders rows r, r + N, ... (the
    interleave of dist.py / render_multi); ranks 0 and N - 1 (the first and last row sets) are timed on their
    own, the best of `reps` runs each, and the predicted efficiency is frame_ms_1 / (N x the slower rank).
    What it leaves out: the canvas gather over RCCL (66 MB per 1920x1080 frame over xGMI, ~1 ms) and any
    interference between GPUs. seed_of(n, r, i): a seed per run (the GI workload: a photon pass in every run,
    as every rank of a real run traces its own maps). batch_samples: the timed frames' own (a rank of the real run
    renders its rows with the same setting)."""
    import torch
    out = {}
    for n in ns:
        ms = {}
        for r in sorted({0, n - 1}):
            best = None
            for i in range(reps):
                seed = seed_of(n, r, i) if seed_of else 0x5EED
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                renderer.render_into(shard.data_ptr(), row_begin=r, row_end=height, row_stride=n, seed=seed,
                                     batch_samples=batch_samples)
                torch.cuda.synchronize()
                t = 1e3 * (time.perf_counter() - t0)
                best = t if best is None else min(best, t)
            ms[r] = best
        mx = max(ms.values())
        out[str(n)] = {"rank_ms": {str(k): round(v, 3) for k, v in ms.items()}, "max_rank_ms": round(mx, 3),
                       "predicted_efficiency": round(frame_ms_1 / (n * mx), 4)}
    return out


def heartbeat(period_s: float = 60.0) -> None:
    """A progress line on stderr every minute while the bench runs (long profiled runs print nothing else)."""
    import threading
    t0 = time.time()

    def beat():
        while True:
            time.sleep(period_s)
            log("bench: running, %.0f s" % (time.time() - t0))

    threading.Thread(target=beat, daemon=True).start()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gi-steps", type=int, default=1, help="timed GI frames (0: skip the GI line)")
    ap.add_argument("--shipped-steps", type=int, default=3,
                    help="timed frames of the shipped light configuration (0: skip the shipped line)")
    ap.add_argument("--scene", default=DEFAULT_SCENE)
    # camera samples per batch on the resident handle: the whole headline frame (frt_render_params.batch_samples; the
    # engine's own default, 2^23, suits one-shot calls such as render_multi, which allocate per call: DESIGN.md §2)
    ap.add_argument("--batch-samples", type=int, default=1 << 27)
    # the GI frame runs on a handle of its own without an untimed warmup frame, so its level state is allocated
    # inside the timed frame: 2^23 samples per batch (a whole-frame batch allocates ~5 s of driver-cleared memory)
    ap.add_argument("--gi-batch-samples", type=int, default=1 << 23)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-render-multi", action="store_true", help="skip the drop-in entry point timing")
    ap.add_argument("--no-scaling-proxy", action="store_true", help="skip the one-GPU proxy of the N-rank split")
    ap.add_argument("--no-gi-proxy", dest="gi_proxy", action="store_false",
                    help="skip the GI workload's scaling proxy (about 1.75 GI frames)")
    ap.add_argument("--cpu-all-threads", action="store_true",
                    help="also time the reference's pool at os.cpu_count() threads (256 on the GPU box)")
    args = ap.parse_args()
    launch_ranks_if_needed(args)
    heartbeat()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    from fast_ray_tracer_amd import build
    from fast_ray_tracer_amd.dist import gather_canvas, shard_capacity
    from fast_ray_tracer_amd.runtime import GpuRenderer, Scene, render_multi

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    def scene_of(name):
        so = os.path.join(build.SCENE_LIB, name + ".so")
        if rank == 0 and not os.path.exists(so):
            build.build_scene(os.path.join(GOLDEN, "scenes", name + ".c"))
        if world > 1:
            dist.barrier()
        return Scene(so, asset_root=ASSETS)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    scene = scene_of(args.scene)
    H, W = scene.height, scene.width

    # the drop-in entry point, once cold (includes the hiprtc compile of the scene's shadow kernel) and
    # once warm, on device 0 only (rank 0 of a 1-rank run; outside the timed region)
    rm = {}
    if world == 1 and not args.no_render_multi:
        from fast_ray_tracer_amd.runtime import render_multi_phases
        torch.cuda.init()
        for key in ("render_multi_wall_ms", "render_multi_wall_ms_warm"):
            t0 = time.perf_counter()
            render_multi(scene, devices=str(local_rank))
            rm[key] = round(1e3 * (time.perf_counter() - t0), 2)
            rm[key.replace("wall_ms", "phases")] = render_multi_phases()
        # a second process's first render_multi: the scene kernel's code object comes from the on-disk cache
        # the first call wrote (frt_jit.hip), so no hiprtc compile; its phases say where the rest goes
        probe = ("import sys, time, json; sys.path.insert(0, %r); from fast_ray_tracer_amd import build as b; "
                 "from fast_ray_tracer_amd.runtime import Scene, render_multi, jit_cache_stats, render_multi_phases; "
                 "sc = Scene(b.build_scene(%r), asset_root=%r); t0 = time.perf_counter(); "
                 "render_multi(sc, devices=%r); print('RM', 1e3 * (time.perf_counter() - t0), "
                 "jit_cache_stats()['compiles']); print('PH', json.dumps(render_multi_phases()))"
                 % (ROOT, os.path.join(GOLDEN, "scenes", args.scene + ".c"), ASSETS, str(local_rank)))
        # three such processes, one after the other: the median (a fresh process's HIP initialisation varies by box)
        probes = []
        for _ in range(3):
            pr = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, timeout=300)
            lines = [ln.split() for ln in pr.stdout.splitlines() if ln.startswith("RM ")]
            ph = [ln[3:] for ln in pr.stdout.splitlines() if ln.startswith("PH ")]
            if pr.returncode == 0 and lines and ph:
                probes.append((float(lines[-1][1]), int(lines[-1][2]), json.loads(ph[-1])))
        if probes:
            probes.sort(key=lambda x: x[0])
            med = probes[len(probes) // 2]
            rm["render_multi_wall_ms_second_process"] = round(med[0], 2)
            rm["render_multi_wall_ms_second_process_runs"] = [round(x[0], 2) for x in probes]
            rm["render_multi_second_process_compiles"] = max(x[1] for x in probes)
            rm["render_multi_phases_second_process"] = med[2]  # (the median process's phases)
        ndev = torch.cuda.device_count()
        if ndev > 1:  # the in-process multi-GPU path of render_multi (one host thread per device)
            t0 = time.perf_counter()
            render_multi(scene, devices=",".join(str(i) for i in range(ndev)))
            rm["render_multi_all_devices_wall_ms"] = round(1e3 * (time.perf_counter() - t0), 2)
            rm["render_multi_all_devices"] = ndev

    renderer = GpuRenderer(scene, device=local_rank)
    cap = shard_capacity(world, H)
    shard = torch.zeros((cap, W, 4), dtype=torch.float64, device="cuda")

    def frame(r, sh, height, seed=0x5EED, stats=False, batch_samples=None):
        st = r.render_into(sh.data_ptr(), row_begin=rank, row_end=height, row_stride=world,
                           batch_samples=args.batch_samples if batch_samples is None else batch_samples, seed=seed,
                           stats=stats)
        canvas = gather_canvas(sh, rank, world, height)
        return st, canvas

    for _ in range(args.warmup):
        frame(renderer, shard, H)
    sync()

    # timed region: exactly K frames, without per-kernel instrumentation (the engine still checks its
    # error flags every frame and fails the render if one is set)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame(renderer, shard, H)
    sync()
    elapsed = time.perf_counter() - t0

    # one instrumented frame after the timed region: per-kernel HIP-event times on the engine stream and
    # the rays traced per frame (the same every frame: same scene, same seed)
    st, _ = frame(renderer, shard, H, stats=True)
    d = st.as_dict()
    if d["errors"]:
        raise RuntimeError("engine reported errors: %s" % d)
    kernel_ms = dict(d["kernel_ms"])
    launches = dict(d["kernel_launches"])
    traced = (d["primary_rays"] + d["secondary_rays"] + d["shadow_rays"]) * args.steps
    walked_rays = d["primary_rays"] + d["secondary_rays"] + d.get("shadow_rays_walked", d["shadow_rays"])

    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    rays = torch.tensor([float(traced)], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(rays, op=dist.ReduceOp.SUM)
    t_max = float(t.item())
    total_rays = float(rays.item())
    proxy = None
    if world == 1 and not args.no_scaling_proxy:
        proxy = {"headline": scaling_proxy(renderer, shard, H, 1e3 * t_max / args.steps,
                                           batch_samples=args.batch_samples)}
    renderer.close()
    del shard

    # ---- the shipped direct-lighting configuration: cornell_box.yml's own 65 535-row jittered light cache, GI off, at
    # the headline size (each path node draws its own cache rows: statistical parity, tests/test_gpu_stochastic.py and
    # the fixed-seed bit-identity of every shadow stage, tests/test_jit.py) ----
    shipped = None
    if args.shipped_steps > 0 and args.scene == DEFAULT_SCENE:
        sscene = scene_of(SHIPPED_SCENE)
        srend = GpuRenderer(sscene, device=local_rank)
        sshard = torch.zeros((shard_capacity(world, sscene.height), sscene.width, 4), dtype=torch.float64, device="cuda")
        frame(srend, sshard, sscene.height)  # (untimed warmup: level state allocated)
        sync()
        s0 = time.perf_counter()
        for _ in range(args.shipped_steps):
            frame(srend, sshard, sscene.height)
        sync()
        s_elapsed = time.perf_counter() - s0
        sst, _ = frame(srend, sshard, sscene.height, stats=True)
        sd = sst.as_dict()
        if sd["errors"]:
            raise RuntimeError("engine reported errors in the shipped frame: %s" % sd)
        st_t = torch.tensor([s_elapsed], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(st_t, op=dist.ReduceOp.MAX)
        s_ms = 1e3 * float(st_t.item()) / args.shipped_steps
        s_rays = (sd["primary_rays"] + sd["secondary_rays"] + sd["shadow_rays"]) * world
        s_ref = reference_rays(SHIPPED_SCENE)
        shipped = {"workload": SHIPPED_SCENE, "width": sscene.width, "height": sscene.height, "spp": sscene.spp,
                   "steps": args.shipped_steps, "ms_per_step": round(s_ms, 3),
                   "value": round(s_rays / (s_ms * 1e-3) / 1e6, 3), "unit": "Mrays/s",
                   "reference_equivalent_mrays_s": round(s_ref / (s_ms * 1e-3) / 1e6, 3) if s_ref else None,
                   "kernel_ms_per_frame": {k: round(v, 3) for k, v in sd["kernel_ms"].items()},
                   "sub_ms_per_frame": {k: round(v, 3) for k, v in sd.get("sub_ms", {}).items()},
                   "lit_nodes_per_frame": sd.get("lit_nodes"),
                   "shadow_pass": {"tile_pairs": sd.get("shadow_tile_pairs"), "tile_pairs_mixed": sd.get("shadow_tile_mixed"),
                                   "tile_sub_pairs": sd.get("shadow_sub_pairs"),
                                   "tile_sub_pairs_mixed": sd.get("shadow_sub_mixed"),
                                   "shadow_rays_per_frame": sd["shadow_rays"],
                                   "shadow_rays_walked_per_ray": sd.get("shadow_rays_walked")},
                   "data": "reference codegen main.c of scenes/cornell_box as shipped (65535-row jittered light cache, "
                           "camera jitter off) with GI off, at 1920x1080x64"}
        srend.close()
        del sshard

    # ---- GI (configs[4]): fresh photon maps inside every timed frame ----
    gi = None
    if args.gi_steps > 0:
        gscene = scene_of(GI_SCENE)
        gr = GpuRenderer(gscene, device=local_rank)
        gshard = torch.zeros((shard_capacity(world, gscene.height), gscene.width, 4), dtype=torch.float64, device="cuda")
        sync()
        g0 = time.perf_counter()
        gstats = []
        for i in range(args.gi_steps):
            # a new seed per frame: the engine traces new photon maps (frt_frame_stats.photon_pass)
            gst, _ = frame(gr, gshard, gscene.height, seed=0x61000 + i, stats=True, batch_samples=args.gi_batch_samples)
            gstats.append(gst.as_dict())
        sync()
        g_elapsed = time.perf_counter() - g0
        gd = gstats[-1]
        if any(s["errors"] for s in gstats):
            raise RuntimeError("engine reported errors in the GI frame: %s" % gstats)
        g_rays = sum(s["primary_rays"] + s["secondary_rays"] + s["shadow_rays"] + s["gather_rays"] for s in gstats)
        gt = torch.tensor([g_elapsed], dtype=torch.float64, device="cuda")
        gr_t = torch.tensor([float(g_rays)], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(gt, op=dist.ReduceOp.MAX)
            dist.all_reduce(gr_t, op=dist.ReduceOp.SUM)
        gi = {"workload": GI_SCENE, "width": gscene.width, "height": gscene.height, "spp": gscene.spp,
              "steps": args.gi_steps, "ms_per_step": round(1e3 * float(gt.item()) / args.gi_steps, 2),
              "value": round(float(gr_t.item()) / float(gt.item()) / 1e6, 3),
              "unit": "Mrays/s (primary+secondary+shadow+final-gather)",
              "photon_pass_in_timed_region": all(s["photon_pass"] for s in gstats),
              "photon_ms": round(gd["photon_ms"], 2), "photons": gd["photons"],
              "gather_rays_per_frame": gd["gather_rays"],
              "kernel_ms_per_frame": {k: round(v, 3) for k, v in gd["kernel_ms"].items()},
              "data": "reference codegen main.c of scenes/cornell_box as shipped (GI on, 65535-row light cache, "
                      "jitter off) with the camera at 1920x1080x64; statistical parity (tests/test_gpu_stochastic.py)"}
        if world == 1 and not args.no_scaling_proxy and proxy is not None and args.gi_proxy:
            proxy["gi"] = scaling_proxy(gr, gshard, gscene.height, gi["ms_per_step"], reps=1,
                                        seed_of=lambda n, r, i: 0x62000 + 16 * n + r,
                                        batch_samples=args.gi_batch_samples)
        if gd.get("sub_launches", {}).get("k_gather_est"):
            gi["gather_est"] = {"ms_per_frame": round(gd["sub_ms"]["k_gather_est"], 3),
                                "launches": gd["sub_launches"]["k_gather_est"],
                                "hit_ms_per_frame": round(gd["sub_ms"].get("k_gather_hit", 0.0), 3)}
            gi["roofline_gather_est"] = gather_roofline(gd)
        gr.close()

    if rank == 0:
        ms_per_step = 1e3 * t_max / args.steps
        value = total_rays / t_max / 1e6
        ref_rays = reference_rays(args.scene)
        roof = frame_roofline(d, kernel_ms, launches, args.scene)
        roof_shadow = shadow_roofline(d, kernel_ms, launches, args.scene) if launches.get("shadow") else None
        out = {
            "metric": "Mrays/s (primary+shadow+secondary) + wall-clock/frame, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("reference codegen main.c of scenes/cornell_box (GI off, 1-row light cache) at 1920x1080, "
                     "8x8 CMJ" if args.scene == DEFAULT_SCENE
                     else "reference codegen main.c: tests/golden/scenes/%s.c" % args.scene),
            "config": {"workload": args.scene, "width": W, "height": H, "spp": scene.spp,
                       "path_length": 5, "parallelism": "rows%d" % world, "batch_samples": args.batch_samples},
            "rays_per_frame_traced": total_rays / args.steps,
            # rays walked one by one (primary + secondary + the shadow rays of the pairs the pair kernels could
            # not decide): `value` counts every shadow ray, also those decided for a whole beam at once
            "rays_per_frame_walked": walked_rays,
            "lit_nodes_per_frame": d.get("lit_nodes"),
            "walked_mrays_s": round(walked_rays * world * args.steps / t_max / 1e6, 3),
            "reference_equivalent_rays_per_frame": ref_rays,
            "reference_equivalent_mrays_s": round(ref_rays * args.steps / t_max / 1e6, 3) if ref_rays else None,
            "kernel_ms_per_frame": {k: round(v, 4) for k, v in kernel_ms.items()},
            "sub_ms_per_frame": {k: round(v, 4) for k, v in d.get("sub_ms", {}).items()},
            "shadow_pass": {
                "kernels_ms_per_frame": {k: round(v, 4) for k, v in d.get("sub_ms", {}).items()
                                         if k.startswith("frt_jit_")},
                "shadow_rays_per_frame": d["shadow_rays"],
                "shadow_rays_walked_per_ray": d.get("shadow_rays_walked"),
                "tile_pairs": d.get("shadow_tile_pairs"), "tile_pairs_mixed": d.get("shadow_tile_mixed"),
                "tile_sub_pairs": d.get("shadow_sub_pairs"), "tile_sub_pairs_mixed": d.get("shadow_sub_mixed"),
                "subtile_pairs": d.get("shadow_subtile_pairs"), "subtile_pairs_mixed": d.get("shadow_subtile_mixed"),
                "node_pairs": d.get("shadow_pairs"), "node_pairs_mixed": d.get("shadow_pairs_mixed"),
                # the fraction of all shadow rays walked one by one (those of the (node, light part) pairs left
                # mixed after the tile and node pair kernels)
                "rays_walked_frac": (round(d["shadow_rays_walked"] / d["shadow_rays"], 4)
                                     if d.get("shadow_rays") else None),
                "note": "every shadow ray's occlusion is computed exactly (bit-identical to a per-ray walk, "
                        "tests/test_jit.py) by a hierarchy of beams: frt_jit_tile (64 consecutive path nodes, 16-sample "
                        "light part), frt_jit_sub (the tile pairs left, per light sample), frt_jit_subtile (the tile "
                        "sample pairs left, per 16-node sub-tile), frt_jit_beam (frt_jit_beam_list: the nodes of the "
                        "sub-tile pairs left), each deciding its beam by interval bounds over all its rays; "
                        "frt_jit_shadow walks the rays left one by one (DESIGN.md 3.3)"},
            "roofline": roof,
            "roofline_shadow_pass": roof_shadow,
        }
        out.update(rm)
        if shipped is not None:
            out["shipped"] = shipped
        if gi is not None:
            out["gi"] = gi
        if proxy is not None:
            proxy["note"] = ("one GPU timing the row sets ranks 0 and N-1 of an N-rank run render (bench.py "
                             "scaling_proxy); predicted_efficiency = the N=1 frame / (N x the slower rank); the RCCL "
                             "canvas gather (~1 ms per 1920x1080 frame) is not included")
            out["scaling_proxy"] = proxy
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(all_threads=args.cpu_all_threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
