"""bench.py's roofline pairing (CPU): a committed PMC summary is divided by a live launch time only when it was
measured on this tree's device sources and its rocprof launch time agrees with the live one (bench.latest_pmc);
otherwise the roofline fields are null with the reason, never a rate from another build or workload."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

W = "cornell_direct_1920x1080_8x8"


def _stats(ms_per_frame=8.8, launches=2):
    d = {"sub_ms": {"k_shade_lit": ms_per_frame}, "sub_launches": {"k_shade_lit": launches}, "shadow_jit": 1}
    return d, {"prepare": 1.0}, {"prepare": 1}


def _pmc(tmp_path, name, avg_ms, sha=None, **extra):
    t = {"kernel": "k_shade_lit", "workload": W, "rocprof_avg_ms": avg_ms,
         "device_source_sha16": sha if sha is not None else bench.device_source_sha(),
         "SQ_INSTS_VALU_ADD_F64_per_launch": 2.5e8, "SQ_INSTS_VALU_MUL_F64_per_launch": 6.3e8,
         "SQ_INSTS_VALU_FMA_F64_per_launch": 2.6e8, "SQ_INSTS_VALU_TRANS_F64_per_launch": 7e7,
         "SQ_INSTS_VALU_per_launch": 2.0e9, "SQ_INSTS_SALU_per_launch": 1.2e9,
         "fetch_size_bytes_per_launch": 6e8, "write_size_bytes_per_launch": 1e9}
    t.update(extra)
    (tmp_path / name).write_text(json.dumps(t))


def test_mismatched_launch_time_gives_null(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "PROFILES", str(tmp_path))
    _pmc(tmp_path, "r06_pmc_k_shade_lit.json", avg_ms=8.8)  # live: 4.4 ms per launch, the PMC twice that
    roof = bench.frame_roofline(*_stats(), W)
    assert roof["kernel"] == "k_shade_lit"
    assert roof["frac"] is None and roof["achieved"] is None and roof["traffic"] is None
    assert "more than 20 % apart" in roof["pmc_rejected"]


def test_other_device_sources_give_null(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "PROFILES", str(tmp_path))
    _pmc(tmp_path, "r06_pmc_k_shade_lit.json", avg_ms=4.4, sha="0123456789abcdef")
    roof = bench.frame_roofline(*_stats(), W)
    assert roof["frac"] is None and "other device sources" in roof["pmc_rejected"]
    _pmc(tmp_path, "r01_pmc_k_shade_lit.json", avg_ms=4.4, sha="")  # (a summary without a hash: rejected too)
    assert bench.latest_pmc("k_shade_lit", W, 4.4, str(tmp_path))[0] is None


def test_matching_pmc_is_used_and_recomputable(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "PROFILES", str(tmp_path))
    _pmc(tmp_path, "r05_pmc_k_shade_lit.json", avg_ms=4.4, sha="0123456789abcdef")  # older, stale
    _pmc(tmp_path, "r06_pmc_k_shade_lit.json", avg_ms=4.0)  # within 20 % of the live 4.4 ms
    roof = bench.frame_roofline(*_stats(), W)
    assert roof["source"].endswith("r06_pmc_k_shade_lit.json") and "pmc_rejected" not in roof
    flops = 64.0 * (2.5e8 + 6.3e8 + 7e7) + 128.0 * 2.6e8
    assert abs(roof["achieved"] - flops / 4.4e-3 / 1e12) < 1e-3
    assert 0 < roof["frac"] <= 1 and roof["bound"] == "valu-fp64"
    assert roof["traffic"] == round(1.6e9)
    assert roof["issue"]["valu"]["frac"] <= 1 and roof["issue"]["salu"]["frac"] <= 1


def test_committed_profiles_all_carry_the_pairing_fields():
    """Every round-6 PMC summary names its workload and kernel, and carries its source hash and rocprof time."""
    import glob
    for p in glob.glob(os.path.join(ROOT, "profiles", "r06*_pmc_*.json")):
        t = json.load(open(p))
        for k in ("kernel", "workload", "device_source_sha16", "rocprof_avg_ms"):
            assert k in t, (p, k)
