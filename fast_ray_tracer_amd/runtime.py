"""ctypes bindings for the frt-mi355x host and device libraries.

A scene is a codegen main.c (``yaml_parser.py scene.yml > main.c``) compiled
unchanged in capture mode (``build.build_scene``): running its ``main`` builds
the scene through the drop-in C API and hands the Camera / World to
``frt_capture_render_multi`` instead of rendering. ``GpuRenderer`` then
flattens the captured scene once, uploads it to HBM and renders rows with the
HIP engine (``include/frt_device.h``). There is no CPU fallback: if
libfrt_device.so or a GPU is missing, construction raises.
"""
from __future__ import annotations

import ctypes
import os
import weakref
import threading

import numpy as np

from . import build

_lock = threading.Lock()
_host = None


class FrameParams(ctypes.Structure):
    _fields_ = [("row_begin", ctypes.c_int64), ("row_end", ctypes.c_int64), ("row_stride", ctypes.c_int64),
                ("seed", ctypes.c_uint64), ("batch_samples", ctypes.c_int64),
                ("count_reference_rays", ctypes.c_int32), ("pad", ctypes.c_int32)]


class FrameStats(ctypes.Structure):
    _fields_ = [("primary_rays", ctypes.c_uint64), ("secondary_rays", ctypes.c_uint64),
                ("shadow_rays", ctypes.c_uint64), ("pruned_secondary", ctypes.c_uint64),
                ("hits", ctypes.c_uint64), ("errors", ctypes.c_uint64), ("render_ms", ctypes.c_double),
                ("kernel_ms", ctypes.c_double * 8), ("kernel_launches", ctypes.c_uint64 * 8),
                ("shadow_kernel_bytes", ctypes.c_double), ("gather_rays", ctypes.c_uint64),
                ("photons", ctypes.c_uint64 * 2), ("photon_ms", ctypes.c_double),
                ("shadow_jit", ctypes.c_int32), ("photon_pass", ctypes.c_int32),
                ("sub_ms", ctypes.c_double * 16), ("sub_launches", ctypes.c_uint64 * 16),
                ("shadow_rays_walked", ctypes.c_uint64), ("shadow_tile_pairs", ctypes.c_uint64),
                ("shadow_tile_mixed", ctypes.c_uint64), ("shadow_pairs", ctypes.c_uint64),
                ("shadow_pairs_mixed", ctypes.c_uint64), ("shadow_sub_pairs", ctypes.c_uint64),
                ("shadow_sub_mixed", ctypes.c_uint64), ("shadow_subtile_pairs", ctypes.c_uint64),
                ("shadow_subtile_mixed", ctypes.c_uint64), ("lit_nodes", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        names = ["trace", "shadow", "shade", "combine", "resolve", "trace_primary", "prepare", "gi"]
        subs = ["frt_jit_beam", "frt_jit_shadow", "k_gather_est", "k_gather_hit", "frt_jit_tile", "frt_jit_sub",
                "frt_jit_subtile", "k_shade_lit", "k_lit_sort"]
        return {
            "primary_rays": int(self.primary_rays), "secondary_rays": int(self.secondary_rays),
            "shadow_rays": int(self.shadow_rays), "pruned_secondary": int(self.pruned_secondary),
            "hits": int(self.hits), "errors": int(self.errors), "render_ms": float(self.render_ms),
            "shadow_kernel_bytes": float(self.shadow_kernel_bytes),
            "gather_rays": int(self.gather_rays), "photons": [int(self.photons[0]), int(self.photons[1])],
            "photon_ms": float(self.photon_ms), "shadow_jit": int(self.shadow_jit),
            "photon_pass": int(self.photon_pass),
            "kernel_ms": {names[i]: float(self.kernel_ms[i]) for i in range(8) if self.kernel_launches[i]},
            "kernel_launches": {names[i]: int(self.kernel_launches[i]) for i in range(8) if self.kernel_launches[i]},
            "sub_ms": {subs[i]: float(self.sub_ms[i]) for i in range(len(subs)) if self.sub_launches[i]},
            "sub_launches": {subs[i]: int(self.sub_launches[i]) for i in range(len(subs)) if self.sub_launches[i]},
            "shadow_rays_walked": int(self.shadow_rays_walked),
            "shadow_tile_pairs": int(self.shadow_tile_pairs), "shadow_tile_mixed": int(self.shadow_tile_mixed),
            "shadow_pairs": int(self.shadow_pairs), "shadow_pairs_mixed": int(self.shadow_pairs_mixed),
            "shadow_sub_pairs": int(self.shadow_sub_pairs), "shadow_sub_mixed": int(self.shadow_sub_mixed),
            "shadow_subtile_pairs": int(self.shadow_subtile_pairs),
            "shadow_subtile_mixed": int(self.shadow_subtile_mixed), "lit_nodes": int(self.lit_nodes),
        }


def host_lib(auto_build: bool = False) -> ctypes.CDLL:
    """Load libfrt_host.so (which pulls in libfrt_device.so) with global symbols."""
    global _host
    with _lock:
        if _host is not None:
            return _host
        if auto_build:
            build.build_host()
        if not os.path.exists(build.HOST_LIB) or not os.path.exists(build.DEVICE_LIB):
            raise RuntimeError("frt native libraries are not built: run __graft_entry__.build() "
                               "(expected %s and %s)" % (build.HOST_LIB, build.DEVICE_LIB))
        lib = ctypes.CDLL(build.HOST_LIB, mode=ctypes.RTLD_GLOBAL)
        vp = ctypes.c_void_p
        lib.frt_captured.restype = ctypes.c_int
        for fn in ("frt_captured_camera", "frt_captured_world"):
            getattr(lib, fn).restype = vp
        for fn in ("frt_captured_usteps", "frt_captured_vsteps"):
            getattr(lib, fn).restype = ctypes.c_size_t
        lib.frt_captured_jitter.restype = ctypes.c_int
        lib.frt_camera_hsize.restype = ctypes.c_size_t
        lib.frt_camera_hsize.argtypes = [vp]
        lib.frt_camera_vsize.restype = ctypes.c_size_t
        lib.frt_camera_vsize.argtypes = [vp]
        lib.frt_host_prepare.restype = vp
        lib.frt_host_prepare.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_bool, ctypes.c_int]
        lib.frt_host_last_error.restype = ctypes.c_char_p
        lib.frt_device_count.restype = ctypes.c_int
        lib.frt_last_error.restype = ctypes.c_char_p
        lib.frt_render_rows.restype = ctypes.c_int
        lib.frt_render_rows.argtypes = [vp, ctypes.POINTER(FrameParams), vp, ctypes.POINTER(FrameStats)]
        lib.frt_render_rows_device.restype = ctypes.c_int
        lib.frt_render_rows_device.argtypes = [vp, ctypes.POINTER(FrameParams), vp, ctypes.POINTER(FrameStats)]
        lib.frt_scene_release.argtypes = [vp]
        lib.frt_encode_ppm.restype = ctypes.c_size_t
        lib.frt_encode_ppm.argtypes = [vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, vp, ctypes.c_size_t]
        lib.frt_frame_stats_size.restype = ctypes.c_size_t
        if lib.frt_frame_stats_size() != ctypes.sizeof(FrameStats):  # (a stale library against this mirror)
            raise RuntimeError("frt: frt_frame_stats is %d bytes in %s, runtime.py FrameStats %d: rebuild"
                               % (lib.frt_frame_stats_size(), build.DEVICE_LIB, ctypes.sizeof(FrameStats)))
        _host = lib
        return lib


class Scene:
    """A scene built by running a capture-mode generated main.c."""

    def __init__(self, scene_so: str, asset_root: str | None = None):
        lib = host_lib()
        self._so = ctypes.CDLL(scene_so, mode=ctypes.RTLD_GLOBAL)
        self._so.frt_scene_main.restype = ctypes.c_int
        cwd = os.getcwd()
        lib.frt_reset_libc_rng()
        try:
            if asset_root:
                os.chdir(asset_root)
            rc = self._so.frt_scene_main()
        finally:
            os.chdir(cwd)
        if rc != 0 or not lib.frt_captured():
            raise RuntimeError("scene main() did not reach render_multi (rc=%d): %s" % (rc, scene_so))
        self.camera = lib.frt_captured_camera()
        self.world = lib.frt_captured_world()
        self.usteps = int(lib.frt_captured_usteps())
        self.vsteps = int(lib.frt_captured_vsteps())
        self.jitter = bool(lib.frt_captured_jitter())
        st = (ctypes.c_ushort * 3)()
        lib.frt_captured_drand48(st)
        self.drand48_state = tuple(st)  # glibc drand48 state at the render_multi call (stochastic checks)
        self.width = int(lib.frt_camera_hsize(self.camera))
        self.height = int(lib.frt_camera_vsize(self.camera))
        self.name = os.path.splitext(os.path.basename(scene_so))[0]

    @property
    def spp(self) -> int:
        return self.usteps * self.vsteps


class GpuRenderer:
    """render_multi's device path for one captured scene on one HIP device."""

    def __init__(self, scene: Scene, device: int = 0):
        self.lib = host_lib()
        if self.lib.frt_device_count() <= 0:
            raise RuntimeError("frt: no HIP device visible; the GPU path has no CPU fallback")
        # the handles an earlier render_multi kept hold their device memory until released (GBs for a GI scene)
        release_render_multi()
        self.scene = scene
        self.device = device
        h = self.lib.frt_host_prepare(scene.camera, scene.world, scene.usteps, scene.vsteps, scene.jitter, device)
        if not h:
            raise RuntimeError("frt: scene upload failed: " + self.lib.frt_host_last_error().decode())
        self.handle = h

    def close(self) -> None:
        if getattr(self, "handle", None):
            self.lib.frt_scene_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _params(self, row_begin, row_end, row_stride, seed, batch_samples):
        p = FrameParams()
        p.row_begin = row_begin
        p.row_end = self.scene.height if row_end is None else row_end
        p.row_stride = row_stride
        p.seed = seed
        p.batch_samples = batch_samples
        return p

    @staticmethod
    def rows_in(row_begin, row_end, row_stride) -> int:
        return len(range(row_begin, row_end, row_stride))

    def render(self, row_begin: int = 0, row_end: int | None = None, row_stride: int = 1, seed: int = 0x5EED,
               batch_samples: int = 0, stats: bool = False):
        """Render rows into a host array (rows, width, 4) float64."""
        p = self._params(row_begin, row_end, row_stride, seed, batch_samples)
        n = self.rows_in(p.row_begin, p.row_end, row_stride)
        out = np.zeros((n, self.scene.width, 4), dtype=np.float64)
        st = FrameStats()
        rc = self.lib.frt_render_rows(self.handle, ctypes.byref(p), out.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.byref(st) if stats else None)
        if rc != 0:
            raise RuntimeError("frt render failed: " + self.lib.frt_last_error().decode())
        return (out, st) if stats else out

    def render_into(self, device_ptr: int, row_begin: int = 0, row_end: int | None = None, row_stride: int = 1,
                    seed: int = 0x5EED, batch_samples: int = 0, stats: bool = False):
        """Render rows into device memory (e.g. a torch.cuda tensor's data_ptr())."""
        p = self._params(row_begin, row_end, row_stride, seed, batch_samples)
        st = FrameStats()
        rc = self.lib.frt_render_rows_device(self.handle, ctypes.byref(p), ctypes.c_void_p(device_ptr),
                                             ctypes.byref(st) if stats else None)
        if rc != 0:
            raise RuntimeError("frt render failed: " + self.lib.frt_last_error().decode())
        return st if stats else None


def render_multi(scene: Scene, devices: str | None = None) -> np.ndarray:
    """The drop-in entry point itself: ``render_multi(cam, world, usteps, vsteps, jitter)``
    (host/frt_render.c; reference renderer.c:244) on the captured scene — flatten, upload
    (incl. the scene-specialised kernel's compile), render over the selected devices
    (``FRT_DEVICES`` list, e.g. "0,0"; default every visible GPU), copy to the host canvas.
    Returns the (height, width, 4) canvas; render_multi's failures are logged by it and
    leave the canvas zeroed (the reference has no error return); ``frt_render_multi_error``
    (host/frt_render.c) names the failure, and it raises here."""
    lib = host_lib()
    vp = ctypes.c_void_p
    lib.render_multi.restype = vp
    lib.render_multi.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_bool]
    lib.canvas_free.argtypes = [vp]
    old = os.environ.get("FRT_DEVICES")
    if devices is not None:
        os.environ["FRT_DEVICES"] = devices
    try:
        c = lib.render_multi(scene.camera, scene.world, scene.usteps, scene.vsteps, scene.jitter)
    finally:
        if devices is not None:
            if old is None:
                os.environ.pop("FRT_DEVICES", None)
            else:
                os.environ["FRT_DEVICES"] = old
    # the canvas's array itself, not a copy (a 1920x1080 canvas is 66 MB): the returned array owns the canvas, and
    # canvas_free runs when it is collected (render_multi's array goes back to host/frt_canvas.c's pinned pool)
    try:
        # struct canvas (canvas.h): Color *arr; size_t width, height; ... — read via the helper
        lib.frt_canvas_data.restype = ctypes.POINTER(ctypes.c_double)
        lib.frt_canvas_data.argtypes = [vp]
        ptr = lib.frt_canvas_data(c)
        out = np.ctypeslib.as_array(ptr, shape=(scene.height, scene.width, 4))
        weakref.finalize(out, lib.canvas_free, c)
    except BaseException:
        lib.canvas_free(c)
        raise
    lib.frt_render_multi_error.restype = ctypes.c_char_p
    err = lib.frt_render_multi_error()
    global _release_registered
    if not _release_registered:  # (the kept handles go before the interpreter's teardown, not during it)
        import atexit
        lib.frt_render_multi_release.restype = None
        atexit.register(lib.frt_render_multi_release)
        _release_registered = True
    if err:
        raise RuntimeError("frt: render_multi failed: " + err.decode(errors="replace"))
    return out


_release_registered = False


def release_render_multi() -> None:
    """Release the device handles render_multi keeps between calls (host/frt_render.c frt_render_multi_release:
    the scene, its compiled kernels and level state on every device of the last call). Registered to run at exit."""
    global _release_registered
    lib = host_lib()
    lib.frt_render_multi_release.restype = None
    lib.frt_render_multi_release()
    if not _release_registered:
        import atexit
        atexit.register(lib.frt_render_multi_release)
        _release_registered = True


RENDER_MULTI_PHASES = ("flatten", "upload", "upload.device_select", "upload.scene_buffers", "upload.walk_records_meshes",
                       "upload.jit_source", "upload.jit_code_object", "upload.jit_module_load", "upload.rest",
                       "upload.total", "render_rows_and_copy", "place_rows", "release", "total", "device_warmup",
                       "device_warmup_wait")


def render_multi_phases() -> dict:
    """The phases of this process's last render_multi in ms (host/frt_render.c frt_render_multi_phases):
    flatten, the slowest device's upload and its sub-phases (frt_upload_phases), render incl. the copy to
    host memory, placing the rows into the canvas, release, total."""
    lib = host_lib()
    lib.frt_render_multi_phases.restype = ctypes.c_int
    lib.frt_render_multi_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = (ctypes.c_double * 16)()
    lib.frt_render_multi_phases(out, 16)
    return {k: round(float(v), 3) for k, v in zip(RENDER_MULTI_PHASES, out)}


def cpu_share() -> int:
    """The host CPUs this process may use: the cgroup's CPU quota (cpu.max) when one is set, else the
    CPUs in its affinity mask. On the GPU box os.cpu_count() reports the whole machine (256) while the
    quota per GPU is 16."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def jit_cache_stats() -> dict:
    """Counters of the scene-specialised kernels' code-object cache (include/frt_device.h
    frt_jit_cache_stats) since the library was loaded."""
    lib = host_lib()
    lib.frt_jit_cache_stats.restype = ctypes.c_int
    lib.frt_jit_cache_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = (ctypes.c_int64 * 5)()
    lib.frt_jit_cache_stats(out, 5)
    return dict(zip(("compiles", "disk_hits", "disk_writes", "module_loads", "module_hits"), map(int, out)))


def _flat_scene(scene: Scene):
    """The scene flattened by the host library (frt_flatten_scene); free with frt_flat_scene_free."""
    lib = host_lib()
    vp = ctypes.c_void_p
    lib.frt_flatten_scene.restype = ctypes.c_int
    lib.frt_flatten_scene.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_bool, vp, ctypes.c_char_p,
                                      ctypes.c_size_t]
    lib.frt_flat_scene_free.argtypes = [vp]
    fs = ctypes.create_string_buffer(4096)  # frt_scene (a few hundred bytes)
    err = ctypes.create_string_buffer(512)
    if lib.frt_flatten_scene(scene.camera, scene.world, scene.usteps, scene.vsteps, scene.jitter, fs, err, 512):
        raise RuntimeError("frt: flatten failed: " + err.value.decode())
    return lib, fs


def jit_check(scene: Scene) -> tuple[int, str, str]:
    """Generate and compile (hiprtc, no device needed) the scene-specialised shadow
    kernel frt_scene_upload would use for this scene: (rc, log, source) with rc 0
    compiled, 1 not eligible (generic walk), -1 compile error (include/frt_device.h)."""
    hl, fs = _flat_scene(scene)
    lib = hl
    lib.frt_jit_check.restype = ctypes.c_int
    lib.frt_jit_check.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                  ctypes.c_size_t]
    log = ctypes.create_string_buffer(1 << 16)
    src = ctypes.create_string_buffer(1 << 22)
    try:
        rc = lib.frt_jit_check(fs, log, len(log), src, len(src))
    finally:
        hl.frt_flat_scene_free(fs)
    return rc, log.value.decode(errors="replace"), src.value.decode(errors="replace")


def mesh_check(scene: Scene) -> tuple[int, dict]:
    """The meshes frt_scene_upload would search per lane in BVHs of their own, built
    and checked on the host (include/frt_device.h frt_mesh_check, no device needed):
    (violations, {"meshes", "triangles", "bvh_nodes", "depth"})."""
    hl, fs = _flat_scene(scene)
    lib = hl
    lib.frt_mesh_check.restype = ctypes.c_int
    lib.frt_mesh_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    out = (ctypes.c_int64 * 4)()
    try:
        bad = lib.frt_mesh_check(fs, out, 4)
    finally:
        hl.frt_flat_scene_free(fs)
    return bad, dict(zip(("meshes", "triangles", "bvh_nodes", "depth"), map(int, out)))


def encode_ppm(rgba: np.ndarray, use_scaling: bool = True) -> bytes:
    """16-bit P6 PPM bytes of a (h, w, 3|4) float64 canvas, encoded by the host
    library exactly as write_ppm_file(c, use_scaling, path) writes them."""
    lib = host_lib()
    h, w = rgba.shape[:2]
    buf = np.zeros((h, w, 4), dtype=np.float64)
    buf[:, :, :rgba.shape[2]] = rgba[:, :, :min(4, rgba.shape[2])]
    if rgba.shape[2] == 3:
        buf[:, :, 3] = 0.0
    n = lib.frt_encode_ppm(buf.ctypes.data_as(ctypes.c_void_p), w, h, int(use_scaling), None, 0)
    out = np.zeros(n, dtype=np.uint8)
    lib.frt_encode_ppm(buf.ctypes.data_as(ctypes.c_void_p), w, h, int(use_scaling),
                       out.ctypes.data_as(ctypes.c_void_p), n)
    return out.tobytes()
