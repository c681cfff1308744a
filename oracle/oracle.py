"""TEST INFRASTRUCTURE ONLY — Python binding of the CPU oracle (oracle/frt_oracle.c).

Importable only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg. The oracle renders a captured scene (see
fast_ray_tracer_amd.runtime.Scene) by restating the reference's recursion on
the CPU; it is the checker, never the product.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from fast_ray_tracer_amd import build  # noqa: E402
from fast_ray_tracer_amd.runtime import host_lib  # noqa: E402


class OracleStats(ctypes.Structure):
    _fields_ = [("primary_rays", ctypes.c_uint64), ("secondary_rays", ctypes.c_uint64),
                ("shadow_rays", ctypes.c_uint64), ("zero_weight_secondary", ctypes.c_uint64)]


_lib = None


def oracle_lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        host_lib()
        if not os.path.exists(build.ORACLE_LIB):
            build.build_oracle()
        lib = ctypes.CDLL(build.ORACLE_LIB)
        vp = ctypes.c_void_p
        lib.frt_oracle_render_rows_strided.restype = ctypes.c_int
        lib.frt_oracle_render_rows_strided.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_bool,
                                                       ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                                       vp, ctypes.POINTER(OracleStats)]
        _lib = lib
    return _lib


def render(scene, row_begin: int = 0, row_end: int | None = None, threads: int = 0, stats: bool = False,
           row_stride: int = 1):
    """Render rows row_begin, row_begin + row_stride, ... below row_end of a captured scene on the CPU;
    (rows, width, 4) float64."""
    lib = oracle_lib()
    row_end = scene.height if row_end is None else row_end
    nrows = len(range(row_begin, row_end, row_stride))
    out = np.zeros((nrows, scene.width, 4), dtype=np.float64)
    st = OracleStats()
    threads = threads or min(8, os.cpu_count() or 1)
    # drand48 (pixel jitter, aperture samples) continues from the state the scene's main() left,
    # as in the reference's executable; with one thread the draw order is the reference's
    host_lib().frt_set_drand48((ctypes.c_ushort * 3)(*scene.drand48_state))
    rc = lib.frt_oracle_render_rows_strided(scene.camera, scene.world, scene.usteps, scene.vsteps, scene.jitter,
                                            row_begin, row_end, row_stride, threads,
                                            out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st))
    if rc != 0:
        raise RuntimeError("oracle render failed (rc=%d)" % rc)
    if stats:
        return out, {"primary_rays": st.primary_rays, "secondary_rays": st.secondary_rays,
                     "shadow_rays": st.shadow_rays, "zero_weight_secondary": st.zero_weight_secondary}
    return out
