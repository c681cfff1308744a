#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: photon-map fixture from the reference itself (run in the build container).

The reference build (oracle/build_ref.sh, the real sources under /root/reference) of the scene
pm_cornell_10k (cornell_box with 10k photons per map, caustic and global maps, one thread) runs with
the harness hooks of oracle/ref_harness.c:
  * FRT_REF_PM_DUMP: each map before pm_balance (stored order) and after it (the balanced kd-tree in
    heap order, pm.c:329-373);
  * FRT_REF_PM_QUERIES / FRT_REF_PM_OUT: pm_irradiance_estimate (pm.c:91-156) at seeded query points
    and normals, with the scene's radius, photon count and cone-filter k.
tests/golden/pm_cornell_10k.npz keeps, per map m: kd_m (n x 9: pos, power, theta, phi, plane in heap
order), perm_m (heap position -> stored index, so the stored order is kd_m[argsort(perm_m)]); and
queries (map, pos, normal), expected (irrad, found), params (radius, k, cone_k).

    python tests/golden/make_pm_fixture.py
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

NAME = "pm_cornell_10k"
REC = np.dtype([("pos", "<f8", 3), ("power", "<f8", 3), ("b", "<i4", 3)])


def read_map(path):
    with open(path, "rb") as f:
        n = int(np.frombuffer(f.read(8), dtype="<i8")[0])
        return np.frombuffer(f.read(n * REC.itemsize), dtype=REC)


def make_queries(maps, rng, per_map=1200):
    """Seeded query points: around stored photons (dense and sparse regions), uniform in the maps'
    box, a few far outside; unit normals (the estimate's direction filter)."""
    qs = []
    for m, kd in enumerate(maps):
        pos = kd["pos"]
        lo, hi = pos.min(0), pos.max(0)
        near = pos[rng.integers(0, len(pos), per_map // 2)] + rng.normal(0.0, 0.04, (per_map // 2, 3))
        unif = rng.uniform(lo - 0.05, hi + 0.05, (per_map // 2 - 10, 3))
        far = rng.uniform(-1.0, 1.0, (10, 3)) * 50.0
        p = np.concatenate([near, unif, far])
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
    kd = [read_map("%s_%d_kd.bin" % (prefix, m)) for m in range(2)]
    stored = [read_map("%s_%d_stored.bin" % (prefix, m)) for m in range(2)]
    # heap position -> stored index (photons are distinct records; match on position + power bytes)
    perms = []
    for m in range(2):
        key = {s.tobytes()[:48]: i for i, s in enumerate(stored[m])}
        perms.append(np.array([key[k.tobytes()[:48]] for k in kd[m]], dtype=np.int32))
    rng = np.random.default_rng(20261016)
    qs = make_queries(kd, rng)
    qfile = os.path.join(mg.SCRATCH, NAME + ".queries")
    with open(qfile, "wb") as f:
        f.write(np.int32(len(qs)).tobytes())
        for m, p, n in qs:
            f.write(np.int32(m).tobytes() + np.asarray(p, "<f8").tobytes() + np.asarray(n, "<f8").tobytes())
    ofile = os.path.join(mg.SCRATCH, NAME + ".estimates")
    env = dict(os.environ, FRT_REF_PM_QUERIES=qfile, FRT_REF_PM_OUT=ofile)
    subprocess.run([binary], cwd=mg.REF_COPY, env=env, stdout=subprocess.DEVNULL, check=True)
    res = np.fromfile(ofile, dtype=np.dtype([("irrad", "<f8", 3), ("found", "<i8")]))
    gi = tree_gi(tree)
    out = os.path.join(HERE, NAME + ".npz")
    arrays = {"query_map": np.array([q[0] for q in qs], np.int32),
              "query_pos": np.array([q[1] for q in qs]), "query_normal": np.array([q[2] for q in qs]),
              "irrad": res["irrad"], "found": res["found"],
              "params": np.array([gi["radius"], gi["k"], gi["cone_k"]])}
    for m in range(2):
        arrays["kd_%d" % m] = np.concatenate([kd[m]["pos"], kd[m]["power"], kd[m]["b"].astype(np.float64)], axis=1)
        arrays["perm_%d" % m] = perms[m]
    np.savez_compressed(out, **arrays)
    print(out, [len(k) for k in kd], "queries", len(qs), "found>0", int((res["found"] > 0).sum()),
          "found>=k", int((res["found"] >= gi["k"]).sum()))
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
