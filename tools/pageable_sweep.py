#!/usr/bin/env python3
"""Pageable end-to-end rate of the host API (1080p, full int32 cost tables) against the number
of host copy threads of the engine's bounce ring (MIPGPU_COPY_THREADS), with the ring's own
timing (MIPGPU_STAGE_STATS, printed when the engine is destroyed).  GPU box:
    python tools/pageable_sweep.py [threads ...]   (MAX_BATCH=n: the engine's max_batch, default 128)
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
import numpy as np  # noqa: E402

from mipgpu import MipEngine, pinned_empty  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402

W, H, B, CALLS = 1920, 1080, 128, 8
os.environ["MIPGPU_STAGE_STATS"] = "1"
frames = synth_frames(W, H, B, 0x1080, 0).astype(np.uint16)
for threads in [int(t) for t in sys.argv[1:]] or [8]:
    os.environ["MIPGPU_COPY_THREADS"] = str(threads)
    with MipEngine(W, H, max_batch=int(os.environ.get("MAX_BATCH", B))) as eng:
        out = {"cost": np.empty((B, eng.costs_per_frame), np.int32)}
        out["cost"].fill(0)
        eng.search(frames, out=out)
        t0 = time.perf_counter()
        eng.wait([eng.search_async(frames, out=out) for _ in range(CALLS)][-1])
        fps = CALLS * B / (time.perf_counter() - t0)
        if threads == int((sys.argv[1:] or [8])[0]):
            pf = pinned_empty(frames.shape, np.uint16)
            pf[:] = frames
            po = {"cost": pinned_empty((B, eng.costs_per_frame), np.int32)}
            eng.search(pf, out=po)
            t0 = time.perf_counter()
            eng.wait([eng.search_async(pf, out=po) for _ in range(CALLS)][-1])
            print("page-locked: %.1f frames/s" % (CALLS * B / (time.perf_counter() - t0)), flush=True)
    print("threads %d: pageable %.1f frames/s" % (threads, fps), flush=True)
