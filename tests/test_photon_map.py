"""Photon map parity against the reference's own balanced maps and estimates.

Fixtures (tests/golden/make_pm_fixture.py), each the reference's maps as its pm_balance left them
(heap order, pm.c:329-494), their storage order before it, and 2400 seeded queries with the
reference's pm_irradiance_estimate results (irradiance and photons used, pm.c:91-156):
  * pm_cornell_10k.npz: the cornell box scene with 10k photons per map (caustic, global), radius 0.3,
    k = 50, cone k 1.1;
  * pm_cornell_shipped_250k.npz: the shipped estimate parameters (cornell_box.yml:18-20: k = 200,
    radius 0.1, cone k 1.0, caustics off) over a 250k-photon global map, a third of the queries at the
    densest photons: 560 queries hold more photons in range than the device's per-wave list (768), so
    the list-overflow path of the device estimate (frt_gi.hpp: the filtered second scan, or the
    re-scans when even that overflows) is compared with the reference.

* CPU: the oracle's balance and both forms of its search (oracle/pm_oracle.py) reproduce the
  fixture; frt_pm_balance (the engine's balance, C ABI, host only) reproduces the heap order and the
  split planes of every internal node.
* GPU: frt_pm_estimate (the device's estimate, frt_gi.hpp wave_irradiance_estimate) over all queries:
  the photons used exactly, the irradiance within 1e-9 of the query's largest channel (the sums run in
  another order).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN

FIXTURES = ["pm_cornell_10k", "pm_cornell_shipped_250k"]
# the device's per-wave list of photons in range (frt_engine.hip kGatherEstCap)
DEVICE_LIST_CAP = 768


@pytest.fixture(scope="module", params=FIXTURES)
def fx(request):
    z = np.load(os.path.join(GOLDEN, request.param + ".npz"))
    d = {k: z[k] for k in z.files}
    d["name"] = request.param
    return d


def maps_of(fx):
    return [m for m in (0, 1) if len(fx["kd_%d" % m])]


def stored_order(fx, m):
    """The map's photons in storage order (before pm_balance), as the device receives them: positions,
    powers and the stored direction bytes (theta, phi)."""
    kd = fx["kd_%d" % m]
    order = np.argsort(fx["perm_%d" % m])
    st = kd[order]
    pos, power = np.ascontiguousarray(st[:, 0:3]), np.ascontiguousarray(st[:, 3:6])
    return pos, power, np.ascontiguousarray(st[:, 6:8].astype(np.uint8))


def heap_kd(fx, m):
    """kd rows with a leading unused row 0 (the reference's 1-based heap)."""
    kd = fx["kd_%d" % m]
    return np.concatenate([np.zeros((1, kd.shape[1])), kd])


def internal_nodes(n):
    """Heap nodes whose split plane the search reads (pm.c:172: i < half_stored_photons)."""
    return np.arange(1, max(1, n // 2 - 1))


def test_fixture_shape(fx):
    assert fx["kd_0"].shape[1] == 9 and fx["kd_1"].shape[1] == 9
    assert len(fx["query_pos"]) == len(fx["irrad"]) == len(fx["found"]) == 2400
    radius, k, cone_k = fx["params"]
    # the fixture exercises both regimes: fewer than k photons in range and the heap
    assert (fx["found"] == int(k)).sum() > 300 and ((fx["found"] > 8) & (fx["found"] < int(k))).sum() > 100
    if fx["name"] == "pm_cornell_10k":
        assert (radius, int(k), cone_k) == (0.3, 50, 1.1)
    else:
        # the shipped parameters (cornell_box.yml:18-20), the global map only (caustics off)
        assert (radius, int(k), cone_k) == (0.1, 200, 1.0)
        assert maps_of(fx) == [1] and len(fx["kd_1"]) == 250001  # max_photons + 1 (pm_store)
        # queries past the device list's capacity: the overflow path is compared with the reference
        assert (fx["in_range"] > DEVICE_LIST_CAP).sum() >= 100 and (fx["in_range"] > 1500).sum() >= 10


@pytest.mark.parametrize("m", [0, 1])
def test_oracle_balance_matches_reference(fx, m):
    import pm_oracle
    if m not in maps_of(fx):
        pytest.skip("empty map")
    pos, _, _ = stored_order(fx, m)
    n = len(pos)
    pbal, plane = pm_oracle.balance(np.concatenate([np.zeros((1, 3)), pos]))
    perm = fx["perm_%d" % m]
    assert np.array_equal(pbal[1:] - 1, perm)
    inner = internal_nodes(n)
    assert np.array_equal(plane[inner], fx["kd_%d" % m][inner - 1, 8].astype(np.int64))


@pytest.mark.parametrize("m", [0, 1])
def test_engine_balance_matches_reference(built, fx, m):
    if m not in maps_of(fx):
        pytest.skip("empty map")
    lib = ctypes.CDLL(built.DEVICE_LIB)
    lib.frt_pm_balance.restype = ctypes.c_int
    lib.frt_pm_balance.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    pos, _, _ = stored_order(fx, m)
    n = len(pos)
    heap_of = np.zeros(n, np.int32)
    plane = np.zeros(n + 1, np.int8)
    assert lib.frt_pm_balance(pos.ctypes.data, n, heap_of.ctypes.data, plane.ctypes.data) == 0
    perm = fx["perm_%d" % m]  # heap position h - 1 -> stored index
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(1, n + 1)
    assert np.array_equal(heap_of, inv)
    inner = internal_nodes(n)
    assert np.array_equal(plane[inner].astype(np.int64), fx["kd_%d" % m][inner - 1, 8].astype(np.int64))


def _close(a, b, rtol=1e-9):
    scale = np.maximum(np.abs(b).max(axis=1, keepdims=True), 1e-300)
    return np.abs(a - b) <= rtol * scale


# the device's sums run in another order: 1e-9 of the query's largest channel (north_star: 1e-4)
DEVICE_RTOL = 1e-9


@pytest.mark.parametrize("m", [0, 1])
def test_oracle_estimates_match_reference(fx, m):
    """Both forms of the search on a sample of the queries (pure Python: a sample keeps it fast)."""
    import pm_oracle
    if m not in maps_of(fx):
        pytest.skip("empty map")
    radius, k, cone_k = float(fx["params"][0]), int(fx["params"][1]), float(fx["params"][2])
    kd = heap_kd(fx, m)
    idx = np.nonzero(fx["query_map"] == m)[0]
    if fx["name"] == "pm_cornell_10k":
        pick = list(idx[::12])
    else:  # the densest queries (past the device list), then a spread
        dense = idx[np.argsort(-fx["in_range"][idx], kind="stable")]
        pick = list(dense[:8]) + list(idx[::80])
    for qi in pick:
        x, nrm = fx["query_pos"][qi], fx["query_normal"][qi]
        step = pm_oracle.locate(kd[:, 0:3], kd[:, 8], x, radius, k)
        closed = pm_oracle.selection(kd[:, 0:3], kd[:, 8], x, radius, k)
        assert sorted(step[0]) == sorted(closed[0]) and step[1] == closed[1]
        irr, found = pm_oracle.irradiance_estimate(kd, x, nrm, radius, k, cone_k, sel=closed)
        assert found == fx["found"][qi]
        assert _close(np.array([irr]), fx["irrad"][qi][None, :]).all(), (qi, irr, fx["irrad"][qi])


@pytest.mark.gpu
def test_device_estimates_match_reference(built, fx):
    lib = ctypes.CDLL(built.DEVICE_LIB)
    lib.frt_last_error.restype = ctypes.c_char_p
    lib.frt_pm_estimate.restype = ctypes.c_int
    vp = ctypes.c_void_p
    lib.frt_pm_estimate.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int64, ctypes.c_double,
                                    ctypes.c_int32, ctypes.c_double, vp, vp]
    radius, k, cone_k = float(fx["params"][0]), int(fx["params"][1]), float(fx["params"][2])
    bad = []
    for m in maps_of(fx):
        pos, power, tpb = stored_order(fx, m)
        idx = np.nonzero(fx["query_map"] == m)[0]
        q = np.ascontiguousarray(np.concatenate([fx["query_pos"][idx], fx["query_normal"][idx]], axis=1))
        irrad = np.zeros((len(idx), 3))
        found = np.zeros(len(idx), np.int64)
        rc = lib.frt_pm_estimate(0, pos.ctypes.data, power.ctypes.data, tpb.ctypes.data, len(pos), q.ctypes.data,
                                 len(idx), radius, k, cone_k, irrad.ctypes.data, found.ctypes.data)
        assert rc == 0, lib.frt_last_error()
        assert np.array_equal(found, fx["found"][idx]), (m, np.nonzero(found != fx["found"][idx])[0][:10])
        ok = _close(irrad, fx["irrad"][idx], DEVICE_RTOL).all(axis=1)
        bad += [(m, int(idx[i]), irrad[i].tolist(), fx["irrad"][idx[i]].tolist()) for i in np.nonzero(~ok)[0]]
    assert not bad, (len(bad), bad[:5])


@pytest.mark.gpu
def test_device_estimate_edge_cases(built):
    """No photons, all photons at one point (ties), queries far from every photon, k above the count."""
    lib = ctypes.CDLL(built.DEVICE_LIB)
    lib.frt_pm_estimate.restype = ctypes.c_int
    vp = ctypes.c_void_p
    lib.frt_pm_estimate.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int64, ctypes.c_double,
                                    ctypes.c_int32, ctypes.c_double, vp, vp]
    import pm_oracle

    def run(pos, power, tp, q, radius, k, cone_k):
        irrad = np.zeros((len(q), 3))
        found = np.zeros(len(q), np.int64)
        pos, power, q = (np.ascontiguousarray(a, dtype=np.float64) for a in (pos, power, q))
        tpb = np.ascontiguousarray(tp, dtype=np.uint8)
        assert lib.frt_pm_estimate(0, pos.ctypes.data, power.ctypes.data, tpb.ctypes.data, len(pos), q.ctypes.data,
                                   len(q), radius, k, cone_k, irrad.ctypes.data, found.ctypes.data) == 0
        return irrad, found

    def oracle(pos, power, tp, q, radius, k, cone_k):
        n = len(pos)
        pbal, plane = pm_oracle.balance(np.concatenate([np.zeros((1, 3)), pos]))
        kd = np.zeros((n + 1, 9))
        kd[1:, 0:3] = pos[pbal[1:] - 1]
        kd[1:, 3:6] = power[pbal[1:] - 1]
        kd[1:, 8] = plane[1:]
        # directions: theta / phi chosen so pm_photon_dir gives d (d built from them below)
        kd[1:, 6:8] = tp[pbal[1:] - 1]
        out = [pm_oracle.irradiance_estimate(kd, qq[0:3], qq[3:6], radius, k, cone_k) for qq in q]
        return np.array([o[0] for o in out]), np.array([o[1] for o in out])

    rng = np.random.default_rng(7)
    n = 3000
    pos = rng.uniform(-1.0, 1.0, (n, 3))
    power = rng.uniform(0.0, 1e-3, (n, 3))
    tp = rng.integers(0, 256, (n, 2)).astype(np.float64)
    # many equal photons at one point: binary64 ties (which of them the search keeps is not reproduced;
    # equal records make the estimate independent of it)
    pos[:400], power[:400], tp[:400] = 0.25, 5e-4, (17.0, 101.0)
    q = np.concatenate([rng.uniform(-1.0, 1.0, (40, 3)), rng.normal(size=(40, 3))], axis=1)
    q[:, 3:] /= np.linalg.norm(q[:, 3:], axis=1, keepdims=True)
    q[0, 0:3] = (0.26, 0.25, 0.24)  # at the ties
    q[-1, 0:3] = 40.0  # nothing in range
    for radius, k in ((0.2, 30), (0.5, 5000)):
        irr_d, f_d = run(pos, power, tp, q, radius, k, 1.1)
        irr_o, f_o = oracle(pos, power, tp, q, radius, k, 1.1)
        assert np.array_equal(f_d, f_o)
        assert _close(irr_d, irr_o, DEVICE_RTOL).all()
    # a larger map of distinct powers (70 000 photons)
    m2 = 70000
    pos2 = rng.uniform(-1.0, 1.0, (m2, 3))
    power2 = rng.uniform(0.0, 1e-3, (m2, 3))
    tp2 = rng.integers(0, 256, (m2, 2)).astype(np.float64)
    q2 = q[:6].copy()
    q2[:, 0:3] = pos2[:6] + 0.01
    irr_d, f_d = run(pos2, power2, tp2, q2, 0.2, 40, 1.1)
    irr_o, f_o = oracle(pos2, power2, tp2, q2, 0.2, 40, 1.1)
    assert np.array_equal(f_d, f_o) and (f_d == 40).all()
    assert _close(irr_d, irr_o, DEVICE_RTOL).all()
    # no photons: nothing found, a zero estimate
    irr_d, f_d = run(np.zeros((0, 3)), np.zeros((0, 3)), np.zeros((0, 2)), q[:4], 0.2, 30, 1.1)
    assert (f_d == 0).all() and (irr_d == 0).all()
