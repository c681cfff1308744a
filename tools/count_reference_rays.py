"""Record the rays the reference casts for a scene (primary + secondary incl.
zero-weight + shadow), counted by the CPU oracle, into tests/golden/golden.json.
bench.py uses them to quote reference-equivalent rates next to traced rates."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_scene, GOLDEN
import oracle

path = os.path.join(GOLDEN, "golden.json")
for name in sys.argv[1:]:
    sc = load_scene(name)
    t = time.time()
    _, st = oracle.render(sc, threads=int(os.environ.get("THREADS", "8")), stats=True)
    st = {k: int(v) for k, v in st.items()}
    st["total"] = st["primary_rays"] + st["secondary_rays"] + st["shadow_rays"]
    st["oracle_seconds"] = round(time.time() - t, 2)
    idx = json.load(open(path))
    idx.setdefault(name, {})["reference_rays"] = st
    json.dump(idx, open(path, "w"), indent=1, sort_keys=True)
    print(name, st, flush=True)
