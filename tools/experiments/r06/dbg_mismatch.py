"""Round 6 debugging aid: which CU shapes / positions of one golden configuration differ between
the engine (MIPGPU_LIB) and the oracle.  python tools/experiments/r06/dbg_mismatch.py NAME"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import golden_utils as G  # noqa: E402
import oracle_lib as O  # noqa: E402
from mipgpu import MipEngine, layout  # noqa: E402

for name in sys.argv[1:]:
    fx = G.load(name)
    c = fx["config"]
    frames = G.inputs(fx)
    with MipEngine(c["width"], c["height"], filter=c["filter"], kernel_idx=c["kernel_idx"], max_batch=c["frames"]) as eng:
        out = eng.search(frames)
    for f in range(c["frames"]):
        oc = O.engine_search(frames[f], c["filter"], c["kernel_idx"])
        oc = oc[0] if isinstance(oc, tuple) else oc
        bad = np.nonzero(out["cost"][f] != oc)[0]
        print(name, "frame", f, "mismatches", len(bad), "of", oc.size)
        ent = layout.ctu_entries()
        seen = {}
        for idx in bad:
            ctu, rest = divmod(int(idx), layout.COSTS_PER_CTU)
            k = (int(ent["w"][rest]), int(ent["h"][rest]))
            seen.setdefault(k, []).append((ctu, int(ent["cu"][rest]), int(ent["mode"][rest]), int(ent["x"][rest]), int(ent["y"][rest])))
        for k, v in sorted(seen.items()):
            modes = sorted(set(m for _, _, m, _, _ in v))
            cus = sorted(set((ct, cu, x, y) for ct, cu, _, x, y in v))
            print("  %dx%d: %d entries, %d CUs (first %s), modes %s" % (k[0], k[1], len(v), len(cus), cus[:6], modes))
