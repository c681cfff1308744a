#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden from the REAL reference.

Run in the build container only (needs /root/reference). For every entry of
SCENES it:

  1. loads the reference scene YAML, applies the listed overrides (image size,
     single-row area-light caches, GI off, output path) and writes it to a
     scratch directory;
  2. runs the reference's own codegen (yaml_parser/yaml_parser.py, from a
     scratch copy of /root/reference) to produce main.c, saved as
     tests/golden/scenes/<name>.c (an input fixture: the program the drop-in
     boundary must accept unchanged);
  3. builds the reference renderer around it (oracle/build_ref.sh ->
     oracle/_ref/bin/<name>), runs it, and stores the raw canvas
     (float64, width x height x 3) plus the sha256 of its 16-bit PPM and PNG
     as tests/golden/<name>.npz / golden.json (expected outputs).

Scene assets the scenes load at run time (OBJ meshes, PNG textures) are
copied as data into tests/golden/assets/ with their relative paths, so the
tests run on a machine without /root/reference.
"""
from __future__ import annotations

import copy
import hashlib
import json
import os
import shutil
import subprocess
import sys
import time

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FRT_REFERENCE_DIR", "/root/reference")
SCRATCH = "/tmp/frt_golden"
REF_COPY = os.path.join(SCRATCH, "ref")

STOCHASTIC_SEEDS = [12345, 777, 31337, 4242, 2718]

# name -> (yaml, overrides, golden canvas kind)
#   size: (w, h); steps: (u, v); cache: area-light cache-size; threads: reference pool size
SCENES = {
    "checkered_sphere_200": ("scenes/checkered_sphere/checkered_sphere.yml", {"size": (200, 200)}),
    "checkered_sphere_800": ("scenes/checkered_sphere/checkered_sphere.yml", {"size": (800, 800), "hash_only": True}),
    "bounding_boxes_200x80": ("scenes/bounding_boxes/bounding_boxes.yml", {"size": (200, 80)}),
    "cornell_direct_64_4x4": ("scenes/cornell_box/cornell_box.yml", {"size": (64, 64), "cache": 1, "gi_off": True}),
    "cornell_direct_128_1x1": ("scenes/cornell_box/cornell_box.yml",
                               {"size": (128, 128), "steps": (1, 1), "cache": 1, "gi_off": True}),
    "checkered_cube_160x80": ("scenes/checkered_cube/checkered_cube.yml", {"size": (160, 80)}),
    "checkered_cylinder_120": ("scenes/checkered_cylinder/checkered_cylinder.yml", {"size": (120, 120)}),
    "checkered_torus_120": ("scenes/checkered_torus/checkered_torus.yml", {"size": (120, 120)}),
    "align_check_plane_120": ("scenes/align_check_plane/align_check_plane.yml", {"size": (120, 120)}),
    "group_test_150x50": ("scenes/group_test/group.yml", {"size": (150, 50)}),
    "shadow_glamour_150x60": ("scenes/shadow_glamour_shot/shadow_glamour_shot.yml", {"size": (150, 60), "cache": 1}),
    "test_scene_120": ("scenes/test/test.yml", {"size": (120, 120)}),
    "teapot_low_100": ("scenes/teapot/teapot.yml", {"size": (100, 100)}),
    "area_light_test_100": ("scenes/area_light_test/area_light_test.yml", {"size": (100, 100), "cache": 1}),
    "reflect_refract_160x80": ("scenes/reflect_refract/reflect_refract.yml", {"size": (160, 80)}),
    "bump_map_100": ("scenes/bump_map_test/bump_map_test.yml", {"size": (100, 100)}),
    # nested refraction: a glass sphere (Ni 1.5) holding an air bubble (Ni 1.0000034) -> refractive containers
    "reflect_refract_test_150": ("scenes/reflect_refract_test/test.yml", {"size": (150, 150)}),
    # stochastic camera paths (drand48 in the reference; statistical parity): independent
    # reference runs (default libc RNG state + re-seeded ones) are stored as refs[k]
    "checkered_sphere_jitter_100": ("scenes/checkered_sphere/checkered_sphere.yml",
                                    {"size": (100, 100), "steps": (4, 4), "jitter": True, "threads": 1,
                                     "extra_seeds": STOCHASTIC_SEEDS}),
    # the benchmark scene as shipped (cache-size 65535, light rows drawn with rand()), camera jitter
    # on, small image: statistical parity of the stochastic direct-lighting path (BASELINE cfg3-ii)
    "cornell_shipped_48_4x4": ("scenes/cornell_box/cornell_box.yml",
                               {"size": (48, 48), "steps": (4, 4), "jitter": True, "gi_off": True, "threads": 1,
                                "extra_seeds": STOCHASTIC_SEEDS}),
    # global illumination (photon maps + final gather): the shipped configuration (1M photons,
    # 8x8 gather, k = 200) at 16x16 (main.c only), and statistical goldens: the shipped GI at 24x24,
    # the raw global-map estimate (visualize-photon-map) and the caustic map alone
    "cornell_gi_16": ("scenes/cornell_box/cornell_box.yml", {"size": (16, 16), "no_golden": True}),
    # include-global with photon-count 0: the reference dereferences a NULL photon map; the
    # drop-in refuses it (test_unimplemented_features_fail_loudly)
    "cornell_gi_nomaps_16": ("scenes/cornell_box/cornell_box.yml",
                             {"size": (16, 16), "no_golden": True, "gi": {"photon-count": 0}}),
    "cornell_gi_24": ("scenes/cornell_box/cornell_box.yml",
                      {"size": (24, 24), "threads": 8, "extra_seeds": STOCHASTIC_SEEDS, "gi": {}}),
    "cornell_gi_visualize_32": ("scenes/cornell_box/cornell_box.yml",
                                {"size": (32, 32), "steps": (2, 2), "threads": 8, "extra_seeds": STOCHASTIC_SEEDS,
                                 "ill": {"visualize-photon-map": True},
                                 "gi": {"usteps": 2, "vsteps": 2, "photon-count": 200000}}),
    "cornell_caustics_32": ("scenes/cornell_box/cornell_box.yml",
                            {"size": (32, 32), "steps": (2, 2), "threads": 8, "extra_seeds": STOCHASTIC_SEEDS,
                             "gi": {"include-caustics": True, "include-final-gather": False,
                                    "photon-count": 100000}}),
    "checkered_sphere_dof_100": ("scenes/checkered_sphere/checkered_sphere.yml",
                                 {"size": (100, 100), "steps": (4, 4), "jitter": True, "threads": 1,
                                  "aperture": (["CIRCULAR_APERTURE", 1.0], 0.4), "extra_seeds": STOCHASTIC_SEEDS}),
    # benchmark scene (BASELINE.json configs[2]: cornell_box 800x800, 4x4 CMJ, full recursion;
    # GI off, single-row area-light cache = the deterministic parity variant). No canvas golden:
    # the reference takes minutes here; parity is checked at the small sizes above.
    "cornell_direct_800_4x4": ("scenes/cornell_box/cornell_box.yml",
                               {"size": (800, 800), "cache": 1, "gi_off": True, "no_golden": True}),
    # bench.py's cpu_baseline sample: the same scene at 200x200 (1/16 of the pixels), the
    # reference's own pthread pool with 16 threads (the GPU box's CPU share)
    "cornell_direct_200_4x4_t16": ("scenes/cornell_box/cornell_box.yml",
                                   {"size": (200, 200), "cache": 1, "gi_off": True, "threads": 16,
                                    "ref_binary_only": True}),
    # ---- round 2 ----
    # the north-star headline: cornell_box at 1920x1080 with an 8x8 CMJ grid (64 spp), deterministic
    # parity variant (GI off, single-row light cache); bench.py's default workload. No canvas golden
    # (the reference needs ~20 min at 16 threads): parity at full size is a row band vs the oracle
    "cornell_direct_1920x1080_8x8": ("scenes/cornell_box/cornell_box.yml",
                                     {"size": (1920, 1080), "steps": (8, 8), "cache": 1, "gi_off": True,
                                      "no_golden": True}),
    # the same camera at 1/64 of the pixels (same 16:9 view, 8x8 CMJ): a canvas golden of the headline
    # configuration and bench.py's cpu_baseline sample (the reference's pthread pool, 16 threads)
    "cornell_direct_240x135_8x8": ("scenes/cornell_box/cornell_box.yml",
                                   {"size": (240, 135), "steps": (8, 8), "cache": 1, "gi_off": True,
                                    "threads": 16}),
    # BASELINE configs[4]: the shipped GI configuration (1M photons, 8x8 final gather) at 1920x1080x64
    "cornell_gi_1920x1080_8x8": ("scenes/cornell_box/cornell_box.yml",
                                 {"size": (1920, 1080), "steps": (8, 8), "no_golden": True}),
    # ---- round 5 ----
    # the direct-lighting frame as shipped (65535-row jittered light cache, camera jitter off as in
    # cornell_box.yml) at the headline size, GI off: bench.py's "shipped" line; parity by row bands through
    # every shadow stage vs the generic walk at a fixed seed (tests/test_jit.py) and by cornell_shipped_48_4x4
    "cornell_shipped_1920x1080_8x8": ("scenes/cornell_box/cornell_box.yml",
                                      {"size": (1920, 1080), "steps": (8, 8), "gi_off": True, "no_golden": True}),
    # GI statistical goldens at 64x64 (round 2: more power than the 24 / 32 px ones)
    "cornell_gi_64": ("scenes/cornell_box/cornell_box.yml",
                      {"size": (64, 64), "threads": 8, "extra_seeds": STOCHASTIC_SEEDS, "gi": {}}),
    "cornell_gi_visualize_64": ("scenes/cornell_box/cornell_box.yml",
                                {"size": (64, 64), "steps": (2, 2), "threads": 8, "extra_seeds": STOCHASTIC_SEEDS,
                                 "ill": {"visualize-photon-map": True},
                                 "gi": {"usteps": 2, "vsteps": 2, "photon-count": 200000}}),
    "cornell_caustics_64": ("scenes/cornell_box/cornell_box.yml",
                            {"size": (64, 64), "steps": (2, 2), "threads": 8, "extra_seeds": STOCHASTIC_SEEDS,
                             "gi": {"include-caustics": True, "include-final-gather": False,
                                    "photon-count": 100000}}),
    # photon-map fixture scene (tests/golden/make_pm_fixture.py): both maps at 10k photons, single thread
    "pm_cornell_10k": ("scenes/cornell_box/cornell_box.yml",
                       {"size": (4, 4), "steps": (1, 1), "threads": 1, "no_golden": True,
                        "gi": {"photon-count": 10000, "include-caustics": True, "include-final-gather": True,
                               "irradiance-estimate-num": 50, "irradiance-estimate-radius": 0.3,
                               "irradiance-estimate-cone-filter-k": 1.1}}),
    # the shipped estimate parameters (cornell_box.yml:18-20: k = 200, radius 0.1, cone 1.0, caustics
    # off) over a 250k-photon global map: dense enough that queries hold more than the device list's
    # 768 photons in range (make_pm_fixture.py)
    "pm_cornell_shipped_250k": ("scenes/cornell_box/cornell_box.yml",
                                {"size": (4, 4), "steps": (1, 1), "threads": 1, "no_golden": True,
                                 "gi": {"photon-count": 250000}}),
    # cfg4 stand-in (bounding_boxes: 6 dragons, BVH) at its 4x4 CMJ grid, small frame
    "bounding_boxes_100x125_4x4": ("scenes/bounding_boxes/bounding_boxes.yml",
                                   {"size": (100, 125), "steps": (4, 4)}),
    # sibenik.yml (cfg4) with the missing sibenik.obj replaced by the textured nave fixture
    # (make_fixture_mesh.py): OBJ+MTL, map_Ka / map_Kd PNG textures through triangle_uv_map,
    # map_bump, smooth (vn) and flat triangles
    "nave_120x150_4x4": ("scenes/sibenik/sibenik.yml",
                         {"size": (120, 150), "steps": (4, 4), "gi_off": True,
                          "define": {"sibenik": {"file": "scenes/frt_nave/nave.obj", "transform": []}},
                          "camera": {"from": [0, 1.7, -3.6], "to": [0, 1.3, 4], "field-of-view": 1.3},
                          "extra_assets": ["scenes/frt_nave/nave.obj", "scenes/frt_nave/nave.mtl",
                                           "scenes/sibenik/mramor6x6.png", "scenes/sibenik/mramor6x6-bump.png",
                                           "scenes/sibenik/KAMEN-stup.png", "scenes/sibenik/kamen.png"]}),
    # (cornell_box_water.yml is not covered: the reference build segfaults while loading
    # CornellBox-Water.obj, so there is nothing to compare against)
    # frt fixture scenes (tests/golden/yml): branches no shipped scene enables
    # (one reference thread: nested_pattern_at_shape writes into the shared primary pattern, a race
    # between the reference's render threads that makes its multi-threaded image irreproducible)
    "patterns_160x80": ("frt:patterns_160x80.yml", {"threads": 1}),
    "circle_light_100": ("frt:circle_light_100.yml", {}),
    "hemisphere_light_100": ("frt:hemisphere_light_100.yml", {}),
    # the other apertures of camera.c:12-82 (dof.yml:14-19), statistical (drand48 in the reference)
    "checkered_sphere_dof_cross_100": ("scenes/checkered_sphere/checkered_sphere.yml",
                                       {"size": (100, 100), "steps": (4, 4), "jitter": True, "threads": 1,
                                        "aperture": (["CROSS_APERTURE", -0.1, 0.1, -0.1, 0.1], 0.4),
                                        "extra_seeds": STOCHASTIC_SEEDS}),
    "checkered_sphere_dof_diamond_100": ("scenes/checkered_sphere/checkered_sphere.yml",
                                         {"size": (100, 100), "steps": (4, 4), "jitter": True, "threads": 1,
                                          "aperture": (["DIAMOND_APERTURE", -1, 1, -1, 1], 0.4),
                                          "extra_seeds": STOCHASTIC_SEEDS}),
    "checkered_sphere_dof_doughnut_100": ("scenes/checkered_sphere/checkered_sphere.yml",
                                          {"size": (100, 100), "steps": (4, 4), "jitter": True, "threads": 1,
                                           "aperture": (["DOUGHNUT_APERTURE", 1.0, 0.5], 0.4),
                                           "extra_seeds": STOCHASTIC_SEEDS}),
    "checkered_sphere_dof_square_100": ("scenes/checkered_sphere/checkered_sphere.yml",
                                        {"size": (100, 100), "steps": (4, 4), "jitter": True, "threads": 1,
                                         "aperture": (["SQUARE_APERTURE"], 0.4), "extra_seeds": STOCHASTIC_SEEDS}),
}
FIXTURE_YML = os.path.join(HERE, "yml")


def find(items, pred):
    return [it for it in items if isinstance(it, dict) and pred(it)]


def apply_overrides(tree, name, ov):
    cams = find(tree, lambda it: it.get("add") == "camera")
    for cam in cams:
        if "size" in ov:
            cam["width"], cam["height"] = ov["size"]
        if "steps" in ov:
            cam["usteps"], cam["vsteps"] = ov["steps"]
            ap = cam.setdefault("aperture", {})
            ap["usteps"], ap["vsteps"] = ov["steps"]
        if "jitter" in ov:
            cam.setdefault("aperture", {})["jitter"] = ov["jitter"]
        if "aperture" in ov:  # (type list, size)
            ap = cam.setdefault("aperture", {})
            ap["type"], ap["size"] = ov["aperture"]
    for cam in cams:
        cam.update(ov.get("camera", {}))
    for name_, fields in ov.get("define", {}).items():
        for d in find(tree, lambda it: it.get("define") == name_):
            d["value"].update(fields)
    if "cache" in ov:
        for light in find(tree, lambda it: it.get("add") == "light" and ("corner" in it or "radius" in it)):
            light["cache-size"] = ov["cache"]
    cfgs = find(tree, lambda it: it.get("add") == "config")
    if not cfgs:
        cfg = {"add": "config"}
        tree.insert(0, cfg)
        cfgs = [cfg]
    cfg = cfgs[0]
    cfg.setdefault("threading", {})["thread-count"] = ov.get("threads", 8)
    cfg.setdefault("output", {})["file"] = os.path.join(SCRATCH, "out", name)
    if "ill" in ov:
        cfg.setdefault("illumination", {}).update(ov["ill"])
    if "gi" in ov:
        cfg.setdefault("illumination", {}).setdefault("global-illumination", {}).update(ov["gi"])
    if ov.get("gi_off"):
        ill = cfg.setdefault("illumination", {})
        ill["include-global"] = False
        ill.setdefault("global-illumination", {})["photon-count"] = 0
    return tree


def sha256(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def assets_of(main_c_text):
    out = set()
    for line in main_c_text.splitlines():
        if "access(\"" in line:
            out.add(line.split("access(\"", 1)[1].split("\"", 1)[0])
    return sorted(out)


def main(names):
    if not os.path.isdir(os.path.join(REF, "src")):
        sys.exit("reference not found at " + REF)
    os.makedirs(os.path.join(SCRATCH, "out"), exist_ok=True)
    if not os.path.isdir(REF_COPY):
        shutil.copytree(REF, REF_COPY)
        subprocess.run(["chmod", "-R", "u+w", REF_COPY], check=True)
    scenes_dir = os.path.join(HERE, "scenes")
    assets_dir = os.path.join(HERE, "assets")
    os.makedirs(scenes_dir, exist_ok=True)
    index_path = os.path.join(HERE, "golden.json")
    index = json.load(open(index_path)) if os.path.exists(index_path) else {}

    for name in names:
        yml_rel, ov = SCENES[name]
        yml_path = (os.path.join(FIXTURE_YML, yml_rel[4:]) if yml_rel.startswith("frt:")
                    else os.path.join(REF_COPY, yml_rel))
        with open(yml_path) as f:
            tree = yaml.safe_load(f)
        for asset in ov.get("extra_assets", []):
            # fixture data the scene loads at run time (our own files or the reference's scene data):
            # into tests/golden/assets and the scratch reference copy the reference binary runs in
            src = os.path.join(assets_dir, asset)
            if not os.path.exists(src):
                os.makedirs(os.path.dirname(src), exist_ok=True)
                shutil.copyfile(os.path.join(REF_COPY, asset), src)
            dst = os.path.join(REF_COPY, asset)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copyfile(src, dst)
        tree = apply_overrides(copy.deepcopy(tree), name, ov)
        yml_out = os.path.join(SCRATCH, name + ".yml")
        with open(yml_out, "w") as f:
            yaml.safe_dump(tree, f, sort_keys=False)
        gen = subprocess.run([sys.executable, "yaml_parser/yaml_parser.py", yml_out], cwd=REF_COPY,
                             capture_output=True, text=True)
        if gen.returncode != 0:
            print("codegen failed for", name, gen.stderr[-2000:])
            continue
        main_c = os.path.join(scenes_dir, name + ".c")
        with open(main_c, "w") as f:
            f.write(gen.stdout)
        for asset in assets_of(gen.stdout):
            dst = os.path.join(assets_dir, asset)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copyfile(os.path.join(REF_COPY, asset), dst)
            mtl = asset[:-3] + "mtl"
            if asset.endswith(".obj") and os.path.exists(os.path.join(REF_COPY, mtl)):
                shutil.copyfile(os.path.join(REF_COPY, mtl), os.path.join(assets_dir, mtl))
        entry = {"yaml": yml_rel, "overrides": {k: v for k, v in ov.items()}}
        if ov.get("no_golden"):
            index[name] = entry
            print(name, "main.c only")
            continue
        b = subprocess.run(["bash", os.path.join(ROOT, "oracle", "build_ref.sh"), main_c, name],
                           capture_output=True, text=True)
        if b.returncode != 0:
            print("reference build failed for", name, b.stderr[-2000:])
            continue
        if ov.get("ref_binary_only"):
            index[name] = entry
            print(name, "main.c + reference binary")
            continue
        binary = b.stdout.strip().splitlines()[-1]
        canvas_bin = os.path.join(SCRATCH, name + ".canvas")
        stats_json = os.path.join(SCRATCH, name + ".stats.json")
        env = dict(os.environ, FRT_REF_CANVAS=canvas_bin, FRT_REF_STATS=stats_json)
        t0 = time.time()
        r = subprocess.run([binary], cwd=REF_COPY, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        if r.returncode != 0:
            print("reference run failed for", name, r.stderr[-2000:])
            continue
        stats = json.load(open(stats_json))
        w, h = stats["width"], stats["height"]
        canvas = np.fromfile(canvas_bin, dtype=np.float64).reshape(h, w, 4)[:, :, :3]
        out_base = os.path.join(SCRATCH, "out", name)
        entry.update({
            "width": w, "height": h, "usteps": stats["usteps"], "vsteps": stats["vsteps"],
            "ref_threads": stats["threads"], "ref_render_multi_seconds": stats["render_multi_seconds"],
            "ppm_sha256": sha256(out_base + ".ppm"), "png_sha256": sha256(out_base + ".png"),
            "canvas_sum": [float(x) for x in canvas.reshape(-1, 3).sum(axis=0)],
        })
        arrays = {"canvas": canvas}
        if ov.get("extra_seeds"):
            # further independent reference renders (drand48 / rand() re-seeded by the harness)
            extra = []
            for sd in ov["extra_seeds"]:
                env2 = dict(env, FRT_REF_DRAND_SEED=str(sd))
                r2 = subprocess.run([binary], cwd=REF_COPY, env=env2, stdout=subprocess.DEVNULL,
                                    stderr=subprocess.PIPE, text=True)
                if r2.returncode != 0:
                    raise RuntimeError("extra reference run failed for %s: %s" % (name, r2.stderr[-2000:]))
                extra.append(np.fromfile(canvas_bin, dtype=np.float64).reshape(h, w, 4)[:, :, :3])
            arrays["refs"] = np.stack([canvas] + extra)
            entry["stochastic"] = True
            if "gi" in ov:
                entry["gi"] = True  # photon maps: statistical parity against the reference renders only
            entry["extra_seeds"] = list(ov["extra_seeds"])
        if not ov.get("hash_only"):
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
            entry["canvas"] = name + ".npz"
        index[name] = entry
        print("%-28s %4dx%-4d %.2fs (wall %.1fs)" % (name, w, h, stats["render_multi_seconds"], time.time() - t0))
        with open(index_path, "w") as f:
            json.dump(index, f, indent=1, sort_keys=True)
    with open(index_path, "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or list(SCENES))
