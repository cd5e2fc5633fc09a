#!/usr/bin/env python3
"""Per-call time of the first calls of a fresh engine (synchronous), then of rounds of 8
queued calls (1080p, page-locked buffers): does a
new engine (or the first use of an output kind) run slow for a while?  Prints one JSON line
per phase: the call times in ms."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mipgpu import MipEngine, pinned_empty  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402

W, H = 1920, 1080
torch.cuda.init()
if os.environ.get("NO_GC"):  # is a spike Python's garbage collector?
    import gc
    gc.disable()
src = synth_frames(W, H, 1, 0x1080, 0)
fr = pinned_empty((1, H, W), np.uint16)
fr[:] = src
with MipEngine(W, H, max_batch=1) as eng:
    n = eng.cus_per_frame
    dec = dict(costs=False, best=True, out={"best_mode": pinned_empty((1, n), np.uint8),
                                            "best_cost": pinned_empty((1, n), np.int32)})
    full = dict(out={"cost": pinned_empty((1, eng.costs_per_frame), np.int32)})
    for phase, kw in (("dec", dec), ("full", full), ("dec2", dec)):
        ts = []
        for _ in range(int(os.environ.get("NCALLS", "40"))):
            t0 = time.perf_counter()
            eng.search(fr, **kw)
            ts.append(round(1e3 * (time.perf_counter() - t0), 3))
        print(json.dumps({"phase": phase, "ms": ts}), flush=True)
    for phase, kw in (("dec_q8", dec), ("full_q8", full)):  # rounds of 8 queued calls
        ts = []
        for _ in range(12):
            t0 = time.perf_counter()
            tk = [eng.search_async(fr, **kw) for _ in range(8)]
            eng.wait(tk[-1])
            ts.append(round(1e3 * (time.perf_counter() - t0), 3))
            del tk
        print(json.dumps({"phase": phase, "ms_per_8": ts}), flush=True)
