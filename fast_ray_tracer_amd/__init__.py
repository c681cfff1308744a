"""frt-mi355x: an MI355X-native (gfx950, HIP) renderer for fast_ray_tracer's
primary-ray -> intersect -> shade_hit path, behind the reference's own
render_multi() / scene-construction C API.

    host/   C11 drop-in scene API (headers at the reference's src/... paths)
    csrc/   hand-written HIP kernels + the C ABI of include/frt_device.h
    runtime ctypes bindings used by tests and bench.py
    build   gcc / hipcc recipes (in-tree shared objects)
"""
from . import build  # noqa: F401

__all__ = ["build"]
