"""Drop-in boundary checks that need no GPU.

* every generated main.c in tests/golden/scenes compiles unchanged against
  the frt headers and links against libfrt_host (the YAML->C pipeline drops in);
* libfrt_device.so loads and exports every function include/frt_device.h declares;
* the CMJ sample tables match the reference's known answers.
"""
import ctypes
import glob
import os
import re
import subprocess

import pytest

from conftest import GOLDEN, ROOT


def declared_functions(header):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(frt_\w+)\s*\(", text)))


def test_device_library_exports_abi(built):
    lib = ctypes.CDLL(built.DEVICE_LIB)
    names = declared_functions(os.path.join(ROOT, "include", "frt_device.h"))
    assert "frt_render_rows" in names and "frt_scene_upload" in names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_frame_stats_layout_matches_runtime_mirror(built):
    """runtime.py's ctypes FrameStats mirrors include/frt_device.h frt_frame_stats: the library reports the struct's
    size as built (frt_frame_stats_size) and the mirror has the same."""
    from fast_ray_tracer_amd.runtime import FrameStats
    lib = ctypes.CDLL(built.DEVICE_LIB)
    lib.frt_frame_stats_size.restype = ctypes.c_size_t
    assert lib.frt_frame_stats_size() == ctypes.sizeof(FrameStats)


def test_device_count_without_gpu_is_safe(built):
    lib = ctypes.CDLL(built.DEVICE_LIB)
    lib.frt_device_count.restype = ctypes.c_int
    assert lib.frt_device_count() >= 0


REFERENCE_API = [
    # functions the codegen emits
    "aperture", "view_transform", "camera", "array_of_lights", "point_light", "hemisphere_light", "area_light",
    "circle_light", "array_of_shapes", "sphere", "plane", "cube", "cone", "cylinder", "toroid", "triangle",
    "smooth_triangle", "csg", "group", "shape_set_transform", "shape_set_material", "shape_set_material_recursive",
    "shape_copy", "construct_group_from_obj_file", "material_alloc", "checker_pattern_alloc",
    "gradient_pattern_alloc", "radial_gradient_pattern_alloc", "ring_pattern_alloc", "stripe_pattern_alloc",
    "blended_pattern_alloc", "nested_pattern_alloc", "perturbed_pattern_alloc", "array_of_patterns",
    "texture_map_pattern", "uv_check_pattern", "uv_align_check_pattern", "uv_texture_pattern", "read_png",
    "pattern_set_transform", "pattern_free", "matrix_translate", "matrix_scale", "matrix_rotate_x", "matrix_rotate_y",
    "matrix_rotate_z", "matrix_shear", "transform_chain", "color_scale", "rgb_to_rgb", "srgb_to_rgb", "xyz_to_rgb",
    "lab_to_rgb", "xyy_to_rgb", "hsl_to_rgb", "world", "array_of_photon_maps", "init_Photon_map", "trace_photons",
    "render_multi", "render", "write_ppm_file", "write_png", "canvas_free",
]


def test_host_library_exports_reference_api(built):
    lib = ctypes.CDLL(built.HOST_LIB, mode=ctypes.RTLD_GLOBAL)
    missing = [n for n in REFERENCE_API if not hasattr(lib, n)]
    assert not missing, missing


@pytest.mark.parametrize("main_c", sorted(glob.glob(os.path.join(GOLDEN, "scenes", "*.c"))))
def test_generated_main_compiles_unchanged(built, tmp_path, main_c):
    """Every generated main.c of the golden set links as an executable against libfrt_host (render_multi on the
    GPU), unchanged."""
    exe = tmp_path / "scene"
    built.build_scene_executable(main_c, str(exe))
    assert exe.exists()


def test_cmj_tables_match_reference_known_answers(built):
    """sampler_2d(false, 4, 4) of the reference (measured)."""
    so = os.path.join(built.LIB, "libfrt_host.so")
    lib = ctypes.CDLL(so)

    class Sampler(ctypes.Structure):
        _fields_ = [("dimensions", ctypes.c_size_t), ("needs_hemi_coords", ctypes.c_bool),
                    ("nt", ctypes.c_double * 4), ("nb", ctypes.c_double * 4),
                    ("steps_by_dimension", ctypes.POINTER(ctypes.c_size_t)), ("arr", ctypes.POINTER(ctypes.c_double)),
                    ("jittered", ctypes.c_bool)]

    expected = {(0, 0): (0.15625, 0.15625), (1, 0): (0.40625, 0.03125), (2, 0): (0.65625, 0.21875),
                (3, 0): (0.90625, 0.09375), (0, 1): (0.03125, 0.40625), (1, 1): (0.28125, 0.28125),
                (2, 1): (0.53125, 0.46875), (3, 1): (0.78125, 0.34375), (0, 2): (0.21875, 0.65625),
                (1, 2): (0.46875, 0.53125), (2, 2): (0.71875, 0.71875), (3, 2): (0.96875, 0.59375),
                (0, 3): (0.09375, 0.90625), (1, 3): (0.34375, 0.78125), (2, 3): (0.59375, 0.96875),
                (3, 3): (0.84375, 0.84375)}
    s = Sampler()
    lib.sampler_2d(ctypes.c_bool(False), ctypes.c_size_t(4), ctypes.c_size_t(4), None, ctypes.byref(s))
    for (u, v), (x, y) in expected.items():
        idx = (ctypes.c_size_t * 2)(u, v)
        res = (ctypes.c_double * 2)()
        lib.sampler_get_point_2d(ctypes.byref(s), idx, res)
        assert (res[0], res[1]) == (x, y), (u, v)
    lib.sampler_2d(ctypes.c_bool(False), ctypes.c_size_t(1), ctypes.c_size_t(1), None, ctypes.byref(s))
    idx = (ctypes.c_size_t * 2)(0, 0)
    res = (ctypes.c_double * 2)()
    lib.sampler_get_point_2d(ctypes.byref(s), idx, res)
    assert (res[0], res[1]) == (0.5, 0.5)


def test_oracle_drop_in_executable_writes_reference_ppm(built, tmp_path):
    """A generated main.c linked against the oracle's render_multi writes the
    reference's PPM bytes (checks scene API + PPM writer end to end)."""
    import hashlib
    import json
    main_c = os.path.join(GOLDEN, "scenes", "checkered_sphere_200.c")
    exe = tmp_path / "cs"
    built.build_scene_executable(main_c, str(exe), oracle=True)
    src = open(main_c).read()
    out_base = re.search(r'global_config.output.file_path = "([^"]+)"', src).group(1)
    os.makedirs(os.path.dirname(out_base), exist_ok=True)
    subprocess.run([str(exe)], cwd=os.path.join(GOLDEN, "assets"), check=True, stdout=subprocess.DEVNULL,
                   env=dict(os.environ, FRT_ORACLE_THREADS="2"))
    idx = json.load(open(os.path.join(GOLDEN, "golden.json")))
    assert hashlib.sha256(open(out_base + ".ppm", "rb").read()).hexdigest() == idx["checkered_sphere_200"]["ppm_sha256"]
    assert hashlib.sha256(open(out_base + ".png", "rb").read()).hexdigest() == idx["checkered_sphere_200"]["png_sha256"]
