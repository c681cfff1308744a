"""The CPU oracle is pinned against the real reference.

tests/golden/*.npz are raw canvases dumped by the reference renderer itself
(oracle/build_ref.sh, tests/golden/make_golden.py). The oracle — a C
restatement of the reference's recursion over the drop-in scene API — must
reproduce them bit for bit, and the host PPM encoder must reproduce the
reference's PPM bytes.
"""
import hashlib

import numpy as np
import pytest

from conftest import canvas_goldens, fresh_scene, golden_index, load_golden_canvas, load_scene


@pytest.mark.parametrize("name", [n for n in canvas_goldens() if not golden_index()[n].get("gi")])
def test_oracle_matches_reference_bit_exact(built, name):
    """(Global-illumination goldens are checked statistically on the GPU only: the oracle
    restates the direct / recursive path, not the photon tracer.)"""
    import oracle
    stochastic = bool(golden_index()[name].get("stochastic"))
    # stochastic goldens (drand48 jitter / apertures, rand() light-cache rows) were rendered by the
    # reference single-threaded, right after its main() built the scene: capture the scene afresh
    # (libc RNG state as the reference had it) and render with one thread to reproduce the draw order
    scene = fresh_scene(name) if stochastic else load_scene(name)
    img = oracle.render(scene, threads=1 if stochastic else 4)[:, :, :3]
    ref = load_golden_canvas(name)
    assert img.shape == ref.shape
    diff = np.abs(img - ref)
    assert np.array_equal(img, ref), f"max |d| = {diff.max():.3e}, {int((diff > 0).sum())} channels differ"


@pytest.mark.parametrize("name", canvas_goldens())
def test_ppm_encoder_matches_reference_bytes(built, name):
    from fast_ray_tracer_amd.runtime import encode_ppm
    ref = load_golden_canvas(name)
    assert hashlib.sha256(encode_ppm(ref)).hexdigest() == golden_index()[name]["ppm_sha256"]


def test_oracle_row_ranges_compose(built):
    """Rendering disjoint row ranges reproduces the full frame (the multi-GPU split contract)."""
    import oracle
    scene = load_scene("cornell_direct_128_1x1")
    full = oracle.render(scene, threads=4)
    top = oracle.render(scene, 0, 40, threads=2)
    bottom = oracle.render(scene, 40, scene.height, threads=2)
    assert np.array_equal(np.concatenate([top, bottom]), full)


def test_oracle_counts_reference_rays(built):
    """Ray accounting of the reference: checkered_sphere casts one
    zero-weight refraction ray and one shadow ray per hit."""
    import oracle
    scene = load_scene("checkered_sphere_200")
    _, st = oracle.render(scene, threads=2, stats=True)
    assert st["primary_rays"] == 200 * 200
    assert st["secondary_rays"] == st["zero_weight_secondary"]
    assert st["shadow_rays"] == st["secondary_rays"]  # one point light, one shadow ray per shaded hit
