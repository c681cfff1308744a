#!/usr/bin/env python3
"""bench.py — frt-mi355x headline benchmark.

Workload (BASELINE.json configs[2]): cornell_box at 800x800 with a 4x4 CMJ
sub-pixel grid (16 spp), full reflection/refraction recursion (path length 5),
one 10x10 area light; GI off and a single-row light cache (the deterministic
parity variant the tests check bit-for-bit against the reference). The scene is
the reference codegen's own main.c (tests/golden/scenes/), built through the
drop-in API in capture mode.

One step = one full frame: every rank renders its interleaved rows on its GPU
(HBM-resident output), then the canvas is gathered on rank 0 over RCCL.
Metric: Mrays/s of rays actually traced (primary + secondary + shadow), summed
over ranks, plus wall-clock per frame; reference-equivalent Mrays/s (the rays the
reference would cast, counted by the oracle: zero-weight secondary subtrees
included) are reported beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scene NAME] [--no-cpu-baseline]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
ASSETS = os.path.join(GOLDEN, "assets")
DEFAULT_SCENE = "cornell_direct_800_4x4"
CPU_SAMPLE_SCENE = "cornell_direct_200_4x4_t16"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
PMC_FILE = "r01_pmc_shadow.json"  # tools/profile_round.sh + profile_summary.py: FETCH/WRITE_SIZE, SQ_* of the shadow kernel
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD per 2 cycles (SIMD32; binary64
# and transcendental instructions take 2-4x: profiles/r01_microbench_valu.txt) at the 2.4 GHz peak clock
VALU_PEAK_GINST_S = 1024 * 2.4 / 2.0

# algorithmic HBM bytes of k_shadow ("byte model"), reported by the engine per frame as
# stats.shadow_kernel_bytes: per shaded path node the 64-byte ShadowHead it reads (over_point,
# key, material; one cache line) and one 4-byte unshadowed count per light it writes. Light points
# and sample tables (a few KB) stay in cache and are not counted.


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(golden_index: dict) -> dict | None:
    """Time the reference's own pthread render_multi (oracle/_ref build) on this host
    on a bounded sample of the same scene."""
    entry = golden_index.get(CPU_SAMPLE_SCENE, {})
    exe = os.path.join(ROOT, "oracle", "_ref", "bin", CPU_SAMPLE_SCENE)
    rays = entry.get("reference_rays", {}).get("total")
    if not os.path.exists(exe) or not rays:
        log("cpu_baseline: reference sample binary or its ray count missing; skipped")
        return None
    stats = "/tmp/frt_bench_ref_stats_%d.json" % os.getpid()
    os.makedirs("/tmp/frt_golden/out", exist_ok=True)
    t0 = time.time()
    proc = subprocess.run([exe], cwd=ASSETS, env=dict(os.environ, FRT_REF_STATS=stats), stdout=subprocess.DEVNULL,
                          stderr=subprocess.PIPE, text=True, timeout=600)
    if proc.returncode != 0:
        log("cpu_baseline: reference run failed:", proc.stderr[-500:])
        return None
    st = json.load(open(stats))
    secs = st["render_multi_seconds"]
    return {"value": round(rays / secs / 1e6, 4), "unit": "Mrays/s", "cores": int(st["threads"]),
            "kind": "reference", "seconds": round(secs, 3), "wall_seconds": round(time.time() - t0, 3),
            "sample": "%s: reference render_multi (pthread pool, %d threads), %dx%dx%d spp, %d reference rays"
                      % (CPU_SAMPLE_SCENE, st["threads"], st["width"], st["height"], st["usteps"] * st["vsteps"], rays)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene", default=DEFAULT_SCENE)
    ap.add_argument("--batch-samples", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))

    from fast_ray_tracer_amd import build
    from fast_ray_tracer_amd.dist import gather_canvas, shard_capacity
    from fast_ray_tracer_amd.runtime import GpuRenderer, Scene

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    main_c = os.path.join(GOLDEN, "scenes", args.scene + ".c")
    scene_so = os.path.join(build.SCENE_LIB, args.scene + ".so")
    if rank == 0 and not os.path.exists(scene_so):
        build.build_scene(main_c)
    if world > 1:
        dist.barrier()

    scene = Scene(scene_so, asset_root=ASSETS)
    renderer = GpuRenderer(scene, device=local_rank)
    H, W = scene.height, scene.width
    cap = shard_capacity(world, H)
    shard = torch.zeros((cap, W, 4), dtype=torch.float64, device="cuda")

    def frame(stats=False):
        st = renderer.render_into(shard.data_ptr(), row_begin=rank, row_end=H, row_stride=world,
                                  batch_samples=args.batch_samples, stats=stats)
        canvas = gather_canvas(shard, rank, world, H)
        return st, canvas

    for _ in range(args.warmup):
        frame()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    # timed region: exactly K frames, without per-kernel instrumentation (the engine still checks its
    # error flags every frame and fails the render if one is set)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame(stats=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # one instrumented frame after the timed region: per-kernel HIP-event times on the engine stream and
    # the rays traced per frame (the same every frame: same scene, same seed)
    st, _ = frame(stats=True)
    d = st.as_dict()
    if d["errors"]:
        raise RuntimeError("engine reported errors: %s" % d)
    kernel_ms = dict(d["kernel_ms"])
    launches = dict(d["kernel_launches"])
    traced = (d["primary_rays"] + d["secondary_rays"] + d["shadow_rays"]) * args.steps

    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    rays = torch.tensor([float(traced)], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(rays, op=dist.ReduceOp.SUM)
    t_max = float(t.item())
    total_rays = float(rays.item())
    last = d

    if rank == 0:
        with open(os.path.join(GOLDEN, "golden.json")) as f:
            gidx = json.load(f)
        ms_per_step = 1e3 * t_max / args.steps
        value = total_rays / t_max / 1e6
        ref_rays = gidx.get(args.scene, {}).get("reference_rays", {}).get("total")
        # dominant kernel: the largest event time of the instrumented frame
        dom = max(kernel_ms, key=kernel_ms.get)
        avg_ms = kernel_ms[dom] / max(1, launches[dom])
        roof = None
        if dom == "shadow":
            kname = "frt_jit_shadow" if last.get("shadow_jit") else "k_shadow"
            bytes_per_frame = last["shadow_kernel_bytes"]  # engine-side byte model (see above)
            per_launch = bytes_per_frame / max(1, launches[dom])
            achieved = per_launch / (avg_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "kernel": kname,
                    "avg_launch_ms": round(avg_ms, 4), "algorithmic_bytes_per_launch": round(per_launch)}
            # HBM bytes and VALU instructions per launch from the committed PMC passes of this kernel
            # on this workload (tools/profile_round.sh); the kernel is VALU-issue bound, not HBM bound:
            # "valu" relates its instruction count to the live kernel time
            pmc = os.path.join(ROOT, "profiles", PMC_FILE)
            if os.path.exists(pmc):
                t = json.load(open(pmc))
                if t.get("kernel") == kname and t.get("workload") == args.scene:
                    roof["traffic"] = round(t["traffic_bytes_per_launch"])
                    roof["traffic_source"] = "profiles/" + PMC_FILE
                    if "SQ_INSTS_VALU_per_launch" in t:
                        ginst = t["SQ_INSTS_VALU_per_launch"] / (avg_ms * 1e-3) / 1e9
                        roof["valu"] = {"achieved": round(ginst, 1), "peak": VALU_PEAK_GINST_S,
                                        "unit": "G wave64 VALU inst/s", "frac": round(ginst / VALU_PEAK_GINST_S, 3),
                                        "valu_inst_per_64_rays": round(t.get("valu_insts_per_wave", 0), 1)}
        else:
            roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                    "traffic": None, "kernel": dom, "avg_launch_ms": round(avg_ms, 4)}
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
            "data": ("reference codegen main.c of scenes/cornell_box (GI off, 1-row light cache)"
                     if args.scene == DEFAULT_SCENE else "reference codegen main.c: tests/golden/scenes/%s.c" % args.scene),
            "config": {"workload": args.scene, "width": W, "height": H, "spp": scene.spp,
                       "path_length": 5, "parallelism": "rows%d" % world},
            "rays_per_frame_traced": total_rays / args.steps,
            "reference_equivalent_rays_per_frame": ref_rays,
            "reference_equivalent_mrays_s": round(ref_rays * args.steps / t_max / 1e6, 3) if ref_rays else None,
            "kernel_ms_per_frame": {k: round(v, 4) for k, v in kernel_ms.items()},
            "roofline": roof,
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(gidx)
        print(json.dumps(out), flush=True)
    renderer.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
