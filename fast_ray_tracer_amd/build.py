"""Build recipes for frt-mi355x (no cmake: plain gcc / hipcc invocations).

Artifacts (all in-tree, git-ignored, shipped to the GPU box with the snapshot):

  fast_ray_tracer_amd/lib/libfrt_device.so   HIP kernels for gfx950 + the C ABI of include/frt_device.h
  fast_ray_tracer_amd/lib/libfrt_host.so     C11 drop-in scene API + render_multi (links libfrt_device)
  fast_ray_tracer_amd/lib/scenes/<name>.so   a generated main.c compiled in capture mode
  oracle/build/liboracle.so                  TEST INFRASTRUCTURE: CPU oracle (checker only)

Host code is compiled with -ffp-contract=off so binary64 arithmetic follows
the reference's ISO-C evaluation (no FMA fusion); device code likewise.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "lib")
SCENE_LIB = os.path.join(LIB, "scenes")
HOST_DIR = os.path.join(PKG, "host")
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_BUILD = os.path.join(ORACLE_DIR, "build")

CONDA_INC = "/opt/conda/include"
CONDA_LIB = "/opt/conda/lib"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CC = os.environ.get("CC", "gcc")
ARCH = os.environ.get("FRT_OFFLOAD_ARCH", "gfx950")

HOST_CFLAGS = ["-std=c11", "-O2", "-fPIC", "-ffp-contract=off", "-D_DEFAULT_SOURCE", "-Wall",
               "-Wno-unused-function", "-I" + HOST_DIR, "-I" + INCLUDE, "-I" + CONDA_INC]

DEVICE_LIB = os.path.join(LIB, "libfrt_device.so")
HOST_LIB = os.path.join(LIB, "libfrt_host.so")
ORACLE_LIB = os.path.join(ORACLE_BUILD, "liboracle.so")


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        sys.stderr.write(proc.stdout + proc.stderr)
        raise RuntimeError("build step failed: " + " ".join(cmd[:4]) + " ...")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_device(force: bool = False) -> str:
    os.makedirs(LIB, exist_ok=True)
    srcs = [os.path.join(CSRC, "frt_engine.hip")]
    deps = srcs + glob.glob(os.path.join(CSRC, "*.hpp")) + [os.path.join(INCLUDE, "frt_device.h")]
    if force or _stale(DEVICE_LIB, deps):
        _run([HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
              "-I" + INCLUDE, "-I" + CSRC, "-o", DEVICE_LIB] + srcs)
    return DEVICE_LIB


def build_host(force: bool = False) -> str:
    build_device(force)
    srcs = sorted(glob.glob(os.path.join(HOST_DIR, "*.c")))
    deps = srcs + glob.glob(os.path.join(HOST_DIR, "**", "*.h"), recursive=True) + [DEVICE_LIB,
                                                                                    os.path.join(INCLUDE, "frt_device.h")]
    if force or _stale(HOST_LIB, deps):
        _run([CC] + HOST_CFLAGS + ["-shared", "-o", HOST_LIB] + srcs +
             ["-L" + LIB, "-lfrt_device", "-L" + CONDA_LIB, "-lpng16", "-lz", "-lm", "-lpthread",
              "-Wl,-rpath,$ORIGIN", "-Wl,-rpath," + CONDA_LIB])
    return HOST_LIB


def build_oracle(force: bool = False) -> str:
    """TEST INFRASTRUCTURE: the CPU oracle (checker), linked against the host scene API."""
    build_host(force)
    os.makedirs(ORACLE_BUILD, exist_ok=True)
    srcs = [os.path.join(ORACLE_DIR, "frt_oracle.c"), os.path.join(ORACLE_DIR, "oracle_render_multi.c")]
    deps = srcs + [os.path.join(ORACLE_DIR, "frt_oracle.h"), HOST_LIB]
    if force or _stale(ORACLE_LIB, deps):
        _run([CC] + HOST_CFLAGS + ["-I" + ORACLE_DIR, "-shared", "-o", ORACLE_LIB] + srcs +
             ["-L" + LIB, "-lfrt_host", "-lm", "-lpthread", "-Wl,-rpath," + LIB])
    return ORACLE_LIB


CAPTURE_DEFINES = ["-Dmain=frt_scene_main", "-Drender_multi=frt_capture_render_multi",
                   "-Dwrite_ppm_file=frt_capture_write_ppm", "-Dwrite_png=frt_capture_write_png"]


def build_scene(main_c: str, name: str | None = None, force: bool = False) -> str:
    """Compile an unmodified generated main.c in capture mode into a shared object."""
    build_host(force)
    os.makedirs(SCENE_LIB, exist_ok=True)
    name = name or os.path.splitext(os.path.basename(main_c))[0]
    out = os.path.join(SCENE_LIB, name + ".so")
    if force or _stale(out, [main_c, HOST_LIB]):
        _run([CC, "-std=c11", "-O1", "-fPIC", "-ffp-contract=off", "-D_DEFAULT_SOURCE", "-w", "-I" + HOST_DIR,
              "-I" + INCLUDE] + CAPTURE_DEFINES + ["-shared", "-o", out, main_c, "-L" + LIB, "-lfrt_host",
                                                  "-Wl,-rpath," + LIB])
    return out


def build_scene_executable(main_c: str, out: str, oracle: bool = False) -> str:
    """The drop-in path: main.c compiled unchanged and linked against libfrt_host
    (render_multi on the GPU), or against the oracle for a CPU port build."""
    build_host()
    cmd = [CC, "-std=c11", "-O1", "-ffp-contract=off", "-D_DEFAULT_SOURCE", "-w", "-I" + HOST_DIR, "-I" + INCLUDE]
    if oracle:
        build_oracle()
        cmd += ["-Drender_multi=frt_oracle_render_multi", "-o", out, main_c, "-L" + ORACLE_BUILD, "-loracle",
                "-Wl,-rpath," + ORACLE_BUILD]
    else:
        cmd += ["-o", out, main_c]
    cmd += ["-L" + LIB, "-lfrt_host", "-Wl,-rpath," + LIB]
    _run(cmd)
    return out


def build_all(force: bool = False) -> None:
    build_device(force)
    build_host(force)
    build_oracle(force)
    for main_c in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "scenes", "*.c"))):
        build_scene(main_c, force=force)
    # the reference build (oracle/_ref) only where its sources exist (this container)
    ref = os.environ.get("FRT_REFERENCE_DIR", "/root/reference")
    if os.path.isdir(os.path.join(ref, "src")) and shutil.which("bash"):
        for main_c in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "scenes", "*.c"))):
            name = os.path.splitext(os.path.basename(main_c))[0]
            target = os.path.join(ORACLE_DIR, "_ref", "bin", name)
            if force or _stale(target, [main_c]):
                _run(["bash", os.path.join(ORACLE_DIR, "build_ref.sh"), main_c, name])


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("ok")
