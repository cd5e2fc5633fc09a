#!/usr/bin/env python3
"""HIP-vs-oracle mismatch census on golden configs (debug aid, GPU box).

usage: python3 tools/diag_mismatch.py CONFIG [CONFIG ...]
For each config: filtered-frame mismatches (defined / undefined samples, first positions)
and cost mismatches (defined / undefined entries, per shape, first CUs with geometry)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import golden_utils as G  # noqa: E402
import oracle_lib as O  # noqa: E402
from mipgpu import MipEngine, layout  # noqa: E402


def main():
    for name in sys.argv[1:] or ["small_alt_2d_float3"]:
        fx = G.load(name)
        c = fx["config"]
        w, h = c["width"], c["height"]
        frames = G.inputs(fx)
        with MipEngine(w, h, filter=c["filter"], kernel_idx=c["kernel_idx"], max_batch=c["frames"]) as eng:
            out = eng.search(frames)
            filt = eng.filter_frames(frames, c["filter"], c["kernel_idx"]) if c["filter"] else None
        e = layout.ctu_entries()
        cols = layout.ctu_grid(w, h)[0]
        for f in range(c["frames"]):
            refs, und, mask = G.refs_and_mask(fx, frames, f)
            print("==", name, "frame", f)
            if filt is not None:
                fb = filt[f] != refs
                print("filtered mismatches: defined %d undefined %d (undefined samples %d)" %
                      ((fb & ~und).sum(), (fb & und).sum(), und.sum()))
                for y, x in np.argwhere(fb)[:8]:
                    print("   y=%d x=%d hip=%d oracle=%d undefined=%d" % (y, x, filt[f][y, x], refs[y, x], und[y, x]))
            oc = O.search(frames[f], refs)
            g = out["cost"][f]
            bad = g != oc
            print("cost mismatches: defined %d undefined %d" % ((bad & mask).sum(), (bad & ~mask).sum()))
            per = {}
            for i in np.nonzero(bad)[0]:
                nm = layout.SHAPES[e["shape"][i % 97840]].name
                per[nm] = per.get(nm, 0) + 1
            print("  per shape", per)
            for i in np.nonzero(bad)[0][:10]:
                ctu, r = divmod(int(i), 97840)
                print("   ctu %d (x0 %d y0 %d) shape %s cu %d x %d y %d mode %d: hip %d oracle %d defined %d" % (
                    ctu, 128 * (ctu % cols), 128 * (ctu // cols), layout.SHAPES[e["shape"][r]].name, e["cu"][r],
                    e["x"][r], e["y"][r], e["mode"][r], g[i], oc[i], mask[i]))


if __name__ == "__main__":
    main()
