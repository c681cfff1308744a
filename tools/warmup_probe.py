"""Where a fresh process's first render_multi goes (round 5): three fresh processes each time the drop-in's first
call with FRT_WARMUP_TRACE=1 (frt_device_warmup's steps on stderr), first alone on the GPU, then while this process
holds most of the GPU's memory (as bench.py's parent does when it starts its second-process probe).
    python tools/warmup_probe.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
PROBE = ("import sys, time, json; sys.path.insert(0, %r); from fast_ray_tracer_amd import build as b; "
         "from fast_ray_tracer_amd.runtime import Scene, render_multi, render_multi_phases; "
         "sc = Scene(b.build_scene(%r), asset_root=%r); t0 = time.perf_counter(); render_multi(sc, devices='0'); "
         "print('RM %%.1f ms' %% (1e3 * (time.perf_counter() - t0))); ph = render_multi_phases(); "
         "print('PH warmup %%.1f upload %%.1f render %%.1f' %% (ph['device_warmup'], ph['upload'], ph['render_rows_and_copy']))"
         % (ROOT, os.path.join(GOLDEN, "scenes", "cornell_direct_1920x1080_8x8.c"), os.path.join(GOLDEN, "assets")))


def run(tag, extra=None):
    for i in range(3):
        p = subprocess.run([sys.executable, "-c", PROBE], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, FRT_WARMUP_TRACE="1", **(extra or {})))
        lines = [ln for ln in (p.stdout + p.stderr).splitlines() if ln.startswith(("RM", "PH", "frt warmup", "frt upload"))]
        print("%s run %d (rc %d): %s" % (tag, i, p.returncode, " | ".join(lines)), flush=True)


run("alone")
import torch  # noqa: E402

torch.cuda.init()
held = torch.empty(int(0.6 * torch.cuda.get_device_properties(0).total_memory) // 8, dtype=torch.float64, device="cuda")
held.fill_(1.0)
torch.cuda.synchronize()
run("parent holding %.0f GB" % (held.numel() * 8 / 1e9))
