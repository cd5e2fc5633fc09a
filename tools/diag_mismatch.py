#!/usr/bin/env python3
"""Per-shape mismatch census of the HIP search vs the C oracle on a golden config (debug aid)."""
import sys, os, numpy as np
sys.path.insert(0, 'vvc-mip-gpu_amd'); sys.path.insert(0, 'tests')
import golden_utils as G, oracle_lib as O
from mipgpu import MipEngine, layout
fx = G.load(sys.argv[1] if len(sys.argv) > 1 else 'small_alt_2d_float3'); c = fx['config']; frames = G.inputs(fx)
with MipEngine(c['width'], c['height'], filter=c['filter'], kernel_idx=c['kernel_idx'], max_batch=c['frames']) as eng:
    out = eng.search(frames)
refs = O.filter_frame(frames[0], c['filter'], c['kernel_idx']) if c['filter'] else None
oc = O.search(frames[0], refs)
g = out['cost'][0]
bad = np.nonzero(g != oc)[0]
print('mismatches', len(bad), 'of', g.size)
per = {}
for i in bad:
    r = i % 97840
    s = max(k for k in range(47) if layout.SHAPES[k].cost_offset <= r)
    per[layout.SHAPES[s].name] = per.get(layout.SHAPES[s].name, 0) + 1
print(per)
for i in bad[:10]: print(i, g[i], oc[i])
