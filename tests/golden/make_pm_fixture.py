#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: photon-map fixture from the reference itself (run in the build container).

The reference build (oracle/build_ref.sh, the real sources under /root/reference) of the scene
pm_cornell_10k (cornell_box with 10k photons per map, caustic and global maps, one thread) runs with
the harness hooks of oracle/ref_harness.c:
  * FRT_REF_PM_DUMP: each map before pm_balance (stored order) and after it (the balanced kd-tree in
    heap order, pm.c:329-373);
  * FRT_REF_PM_QUERIES / FRT_REF_PM_OUT: pm_irradiance_estimate (pm.c:91-156) at seeded query points
    and normals, with the scene's radius, photon count and cone-filter k.
tests/golden/<name>.npz keeps, per map m: kd_m (n x 9: pos, power, theta, phi, plane in heap
order), perm_m (heap position -> stored index, so the stored order is kd_m[argsort(perm_m)]); and
queries (map, pos, normal), expected (irrad, found), params (radius, k, cone_k), in_range (photons
within the radius of each query, counted here in binary64: the fixture-shape tests read the regimes
from it).

Fixtures:
  pm_cornell_10k            10k photons per map (caustic + global), radius 0.3, k = 50, cone 1.1;
  pm_cornell_shipped_250k   the shipped estimate parameters (cornell_box.yml:18-20: k = 200, radius
                            0.1, cone 1.0, caustics off) over a 250k-photon global map; a third of the
                            queries sit at the densest photons, so some hold more photons in range than
                            the device's per-wave list (768, frt_engine.hip kGatherEstCap): its
                            overflow / re-scan path is compared with the reference.

    python tests/golden/make_pm_fixture.py [name]
"""
import copy
import json
import os
import subprocess
import sys

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

NAME = sys.argv[1] if len(sys.argv) > 1 else "pm_cornell_10k"
REC = np.dtype([("pos", "<f8", 3), ("power", "<f8", 3), ("b", "<i4", 3)])


def read_map(path):
    with open(path, "rb") as f:
        n = int(np.frombuffer(f.read(8), dtype="<i8")[0])
        return np.frombuffer(f.read(n * REC.itemsize), dtype=REC)


def densest(pos, radius, count, rng):
    """`count` photons among the densest (most photons within `radius`), a seeded pick."""
    from scipy.spatial import cKDTree
    sample = rng.choice(len(pos), min(len(pos), 40000), replace=False)
    nin = np.array([len(v) for v in cKDTree(pos).query_ball_point(pos[sample], radius)])
    top = sample[np.argsort(-nin, kind="stable")[:count * 4]]
    return pos[rng.choice(top, count, replace=False)]


def make_queries(maps, rng, per_map=1200, dense_frac=0.0, radius=0.3):
    """Seeded query points: around stored photons (dense and sparse regions), uniform in the maps'
    box, a few far outside; unit normals (the estimate's direction filter). dense_frac of them near
    the densest photons (shift below a tenth of the radius)."""
    qs = []
    for m, kd in enumerate(maps):
        pos = kd["pos"]
        if len(pos) == 0:
            continue
        lo, hi = pos.min(0), pos.max(0)
        nd = int(per_map * dense_frac)
        dense = densest(pos, radius, nd, rng) + rng.normal(0.0, 0.1 * radius, (nd, 3)) if nd else np.zeros((0, 3))
        nn = (per_map - nd) // 2
        near = pos[rng.integers(0, len(pos), nn)] + rng.normal(0.0, 0.04, (nn, 3))
        unif = rng.uniform(lo - 0.05, hi + 0.05, (per_map - nd - nn - 10, 3))
        far = rng.uniform(-1.0, 1.0, (10, 3)) * 50.0
        p = np.concatenate([dense, near, unif, far])
        nrm = rng.normal(size=p.shape)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        for i in range(len(p)):
            qs.append((m, p[i], nrm[i]))
    return qs


def main():
    yml_rel, ov = mg.SCENES[NAME]
    os.makedirs(os.path.join(mg.SCRATCH, "out"), exist_ok=True)
    if not os.path.isdir(mg.REF_COPY):
        import shutil
        shutil.copytree(mg.REF, mg.REF_COPY)
        subprocess.run(["chmod", "-R", "u+w", mg.REF_COPY], check=True)
    tree = yaml.safe_load(open(os.path.join(mg.REF_COPY, yml_rel)))
    tree = mg.apply_overrides(copy.deepcopy(tree), NAME, ov)
    yml_out = os.path.join(mg.SCRATCH, NAME + ".yml")
    yaml.safe_dump(tree, open(yml_out, "w"), sort_keys=False)
    gen = subprocess.run([sys.executable, "yaml_parser/yaml_parser.py", yml_out], cwd=mg.REF_COPY,
                         capture_output=True, text=True, check=True)
    main_c = os.path.join(mg.SCRATCH, NAME + ".c")
    open(main_c, "w").write(gen.stdout)
    b = subprocess.run(["bash", os.path.join(mg.ROOT, "oracle", "build_ref.sh"), main_c, NAME],
                       capture_output=True, text=True, check=True)
    binary = b.stdout.strip().splitlines()[-1]
    prefix = os.path.join(mg.SCRATCH, NAME + "_pm")
    env = dict(os.environ, FRT_REF_PM_DUMP=prefix)
    subprocess.run([binary], cwd=mg.REF_COPY, env=env, stdout=subprocess.DEVNULL, check=True)
    kd = [read_map("%s_%d_kd.bin" % (prefix, m)) if os.path.exists("%s_%d_kd.bin" % (prefix, m)) else
          np.zeros(0, REC) for m in range(2)]
    stored = [read_map("%s_%d_stored.bin" % (prefix, m)) if os.path.exists("%s_%d_stored.bin" % (prefix, m)) else
              np.zeros(0, REC) for m in range(2)]
    # heap position -> stored index (photons are distinct records; match on position + power bytes)
    perms = []
    for m in range(2):
        key = {s.tobytes()[:48]: i for i, s in enumerate(stored[m])}
        perms.append(np.array([key[k.tobytes()[:48]] for k in kd[m]], dtype=np.int32))
    rng = np.random.default_rng(20261016)
    gi = tree_gi(tree)
    shipped = NAME != "pm_cornell_10k"
    qs = make_queries(kd, rng, per_map=2400 if shipped else 1200, dense_frac=1.0 / 3.0 if shipped else 0.0,
                      radius=gi["radius"])
    qfile = os.path.join(mg.SCRATCH, NAME + ".queries")
    with open(qfile, "wb") as f:
        f.write(np.int32(len(qs)).tobytes())
        for m, p, n in qs:
            f.write(np.int32(m).tobytes() + np.asarray(p, "<f8").tobytes() + np.asarray(n, "<f8").tobytes())
    ofile = os.path.join(mg.SCRATCH, NAME + ".estimates")
    env = dict(os.environ, FRT_REF_PM_QUERIES=qfile, FRT_REF_PM_OUT=ofile)
    subprocess.run([binary], cwd=mg.REF_COPY, env=env, stdout=subprocess.DEVNULL, check=True)
    res = np.fromfile(ofile, dtype=np.dtype([("irrad", "<f8", 3), ("found", "<i8")]))
    from scipy.spatial import cKDTree
    in_range = np.zeros(len(qs), np.int32)
    for m in range(2):
        sel = [i for i, q in enumerate(qs) if q[0] == m]
        if sel:
            t = cKDTree(kd[m]["pos"])
            in_range[sel] = [len(v) for v in t.query_ball_point(np.array([qs[i][1] for i in sel]), gi["radius"])]
    out = os.path.join(HERE, NAME + ".npz")
    arrays = {"query_map": np.array([q[0] for q in qs], np.int32),
              "query_pos": np.array([q[1] for q in qs]), "query_normal": np.array([q[2] for q in qs]),
              "irrad": res["irrad"], "found": res["found"],
              "params": np.array([gi["radius"], gi["k"], gi["cone_k"]]), "in_range": in_range}
    for m in range(2):
        arrays["kd_%d" % m] = np.concatenate([kd[m]["pos"], kd[m]["power"], kd[m]["b"].astype(np.float64)], axis=1)
        arrays["perm_%d" % m] = perms[m]
    np.savez_compressed(out, **arrays)
    print(out, [len(k) for k in kd], "queries", len(qs), "found>0", int((res["found"] > 0).sum()),
          "found>=k", int((res["found"] >= gi["k"]).sum()), "in_range>768", int((in_range > 768).sum()),
          "max in_range", int(in_range.max()))
    print(json.dumps(gi))


def tree_gi(tree):
    """The scene's estimate parameters as the codegen passes them (yaml_parser config defaults)."""
    src = open(os.path.join(mg.SCRATCH, NAME + ".c")).read()
    def val(field, default):
        tag = "illumination.gi." + field + " = "
        if tag in src:
            return float(src.split(tag, 1)[1].split(";", 1)[0])
        return default
    return {"radius": val("irradiance_estimate_radius", 0.1), "k": int(val("irradiance_estimate_num", 200)),
            "cone_k": val("irradiance_estimate_cone_filter_k", 1.0)}


if __name__ == "__main__":
    main()
