#!/usr/bin/env python3
"""Host-buffer pipeline probe: decisions-only and full-cost end-to-end rates of
mip_search_frames for a few batch sizes (run under rocprofv3 --kernel-trace
--memory-copy-trace to see the overlap of H2D, search, best-mode and D2H)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
import numpy as np  # noqa: E402

from mipgpu import MipEngine, pinned_empty  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402

W, H = 1920, 1080
for B in [int(x) for x in (sys.argv[1:] or ["32"])]:
    host = synth_frames(W, H, min(B, 8), 0x1080, 0)
    hp = pinned_empty((B, H, W), np.uint16)
    for i in range(B):
        hp[i] = host[i % host.shape[0]]
    with MipEngine(W, H, max_batch=B) as eng:
        dout = {"best_mode": pinned_empty((B, eng.cus_per_frame), np.uint8),
                "best_cost": pinned_empty((B, eng.cus_per_frame), np.int32)}
        eng.search(hp, costs=False, best=True, out=dout)
        t0 = time.perf_counter()
        for _ in range(3):
            eng.search(hp, costs=False, best=True, out=dout)
        dec = 3 * B / (time.perf_counter() - t0)
        print("B=%d decisions %.1f frames/s" % (B, dec), flush=True)
