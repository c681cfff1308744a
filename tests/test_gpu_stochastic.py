"""GPU parity for the reference's stochastic paths (statistical).

The reference draws pixel jitter and aperture samples with drand48 and picks
area-light cache rows with rand() % cache_size (sampler.c:411-470,
camera.c:11-90, light.c:196, renderer.c:915). The GPU uses a counter-based
hash of (seed, pixel / sample / path node, draw) instead, so its images are a
different sample of the same distribution: bitwise parity is impossible by
construction (the reference itself is irreproducible multi-threaded). The
goldens hold K = 6 independent reference renders (default libc RNG state and
five re-seeded runs, tests/golden/make_golden.py "extra_seeds"); the oracle
reproduces the first bit for bit (test_oracle_golden.py), which pins what the
distribution is.

Acceptance (distance(gpu, ref) vs distance(ref, ref')),
with four GPU renders (seeds) against the K references:
* mean absolute difference: mean over (gpu, ref) pairs <= 1.15x the mean over
  reference pairs. Pixel noise is heavy-tailed (a few sub-pixel features seen
  by one sample in 16), which makes the RMSE of a single pair unstable; the
  MAD ratio stays within 0.93-1.04 across seed sets (measured against eight
  oracle renders, which reproduce the reference bit for bit per RNG state);
* RMSE: the same ratio <= 1.6 (tail guard);
* image-mean bias within 4 standard errors from the references' spread.
"""
import os

import numpy as np
import pytest

from conftest import golden_index, load_scene

pytestmark = pytest.mark.gpu

STOCHASTIC = sorted(n for n, e in golden_index().items() if e.get("stochastic"))


def _refs(name):
    import os
    from conftest import GOLDEN
    return np.load(os.path.join(GOLDEN, golden_index()[name]["canvas"]))["refs"]


def _rmse(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)))


@pytest.mark.parametrize("name", STOCHASTIC)
def test_gpu_stochastic_paths_match_reference_distribution(built, name):
    from fast_ray_tracer_amd.runtime import GpuRenderer
    refs = _refs(name)
    k = refs.shape[0]
    r = GpuRenderer(load_scene(name))
    gpus = [r.render(seed=sd)[:, :, :3] for sd in (0x5EED, 0xC0FFEE, 11, 12)]
    r.close()
    pairs = [(i, j) for i in range(k) for j in range(i + 1, k)]
    d_ref = np.mean([_rmse(refs[i], refs[j]) for i, j in pairs])
    d_gpu = np.mean([_rmse(g, refs[i]) for g in gpus for i in range(k)])
    a_ref = np.mean([np.abs(refs[i] - refs[j]).mean() for i, j in pairs])
    a_gpu = np.mean([np.abs(g - refs[i]).mean() for g in gpus for i in range(k)])
    m_ref = np.array([x.mean() for x in refs])
    m_gpu = np.array([g.mean() for g in gpus])
    spread = m_ref.std(ddof=1)
    tol = 4 * spread * np.sqrt(1.0 / k + 1.0 / len(gpus)) + 1e-12
    bias = float(m_gpu.mean() - m_ref.mean())
    print(f"{name}: mad(gpu, ref)/mad(ref, ref')={a_gpu / a_ref:.3f} rmse ratio={d_gpu / d_ref:.3f} "
          f"bias={bias:.3e} (tol {tol:.3e})")
    assert d_ref > 0 and a_ref > 0
    assert a_gpu <= 1.15 * a_ref
    assert d_gpu <= 1.6 * d_ref
    assert abs(bias) <= tol


@pytest.mark.parametrize("name", ["checkered_sphere_dof_100", "cornell_caustics_32"])
def test_gpu_stochastic_seeding(built, name):
    """Same seed -> identical image; another seed -> another sample; row splits stay exact
    (photon maps belong to the seed, so they too are reproduced per seed)."""
    from fast_ray_tracer_amd.runtime import GpuRenderer
    r = GpuRenderer(load_scene(name))
    a = r.render(seed=1)
    assert np.array_equal(a, r.render(seed=1))
    assert not np.array_equal(a, r.render(seed=2))
    even, odd = r.render(0, None, 2, seed=1), r.render(1, None, 2, seed=1)
    assert np.array_equal(a[0::2], even) and np.array_equal(a[1::2], odd)
    r.close()


@pytest.mark.gpu
def test_gpu_gi_full_size_row_bands(built):
    """cfg5 at full size (BASELINE configs[4]: the shipped cornell GI configuration at 1920x1080, 8x8 CMJ,
    1M photons, k = 200): two 60-row bands at one seed. Properties: finite; bit-identical on repeat and
    under the 2-way row interleave of a multi-GPU split; and each band's mean within the spread of the
    reference's own renders of the same view. The 1920x1080 camera keeps the 64x64 golden's horizontal
    extent (camera.c: half_width = tan(fov / 2) for aspect >= 1), so 1920-row r lies on 64-row
    14 + r / 30 and a 60-row band starting at a multiple of 30 covers exactly two rows of cornell_gi_64
    (six independent reference renders, each with its own photon maps)."""
    from fast_ray_tracer_amd.runtime import GpuRenderer
    r = GpuRenderer(load_scene("cornell_gi_1920x1080_8x8"))
    refs = np.load(os.path.join(os.path.dirname(__file__), "golden", "cornell_gi_64.npz"))["refs"]
    try:
        for r0 in (240, 600):
            band = r.render(r0, r0 + 60, seed=0x5EED)
            assert band.shape == (60, 1920, 4) and np.isfinite(band).all()
            assert np.array_equal(band, r.render(r0, r0 + 60, seed=0x5EED))
            assert np.array_equal(band[0::2], r.render(r0, r0 + 60, 2, seed=0x5EED))
            assert np.array_equal(band[1::2], r.render(r0 + 1, r0 + 60, 2, seed=0x5EED))
            s0 = 14 + r0 // 30
            ref_means = refs[:, s0:s0 + 2].mean(axis=(1, 2))  # (6, 3)
            mu, sd = ref_means.mean(axis=0), ref_means.std(axis=0, ddof=1)
            got = band[:, :, :3].mean(axis=(0, 1))
            print(f"band {r0}: gpu {got} reference {mu} +- {sd}")
            assert (np.abs(got - mu) <= 4.0 * sd + 0.01 * mu).all(), (r0, got, mu, sd)
    finally:
        r.close()
