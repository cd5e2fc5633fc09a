#!/usr/bin/env python3
"""Does a one-frame full-table engine run slower after something big existed in the process?
Phases, each followed by a fresh max_batch-1 engine's rate for 8 queued one-frame 1080p calls
with page-locked buffers (3 rounds): start; after 6.8 GB of page-locked host buffers were
allocated, touched and freed; after a max_batch-384 engine was created and destroyed; after
both.  One JSON line per phase."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
import numpy as np  # noqa: E402

from mipgpu import MipEngine, pinned_empty  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402

W, H = 1920, 1080


def rate(dec=False):
    fr = pinned_empty((1, H, W), np.uint16)
    fr[:] = synth_frames(W, H, 1, 0x1080, 0)
    with MipEngine(W, H, max_batch=1) as eng:
        n = eng.cus_per_frame
        if dec:
            kw = dict(costs=False, best=True, out={"best_mode": pinned_empty((1, n), np.uint8),
                                                    "best_cost": pinned_empty((1, n), np.int32)})
        else:
            kw = dict(out={"cost": pinned_empty((1, eng.costs_per_frame), np.int32)})
        eng.search(fr, **kw)
        rates = []
        for _ in range(3):
            t0 = time.perf_counter()
            tk = [eng.search_async(fr, **kw) for _ in range(8)]
            eng.wait(tk[-1])
            rates.append(round(8 / (time.perf_counter() - t0), 1))
            del tk
    return rates


fr1 = pinned_empty((1, H, W), np.uint16)
fr1[:] = synth_frames(W, H, 1, 0x1080, 0)


def big_host():
    bufs = [pinned_empty((128 * 1024 * 1024 // 4,), np.int32) for _ in range(int(6.8 * 8))]  # 6.8 GB
    for b in bufs:
        b[::1024] = 1
    del bufs


def big_engine():
    with MipEngine(W, H, max_batch=384):
        pass


def cache():
    from mipgpu import device_cache
    return device_cache(0)


print(json.dumps({"phase": "start", "fps": rate(), "device_cache": cache()}), flush=True)
if os.environ.get("RAW"):  # a plain 20 GB hipMalloc / hipFree in the engine's HIP runtime
    import ctypes
    from mipgpu import hip_runtimes, library
    library()
    hip = ctypes.CDLL(hip_runtimes()[0])
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(20 << 30)) == 0
    print(json.dumps({"phase": "holding a 20 GB hipMalloc", "fps": rate()}), flush=True)
    assert hip.hipFree(p) == 0
    print(json.dumps({"phase": "after freeing it", "fps": rate()}), flush=True)
    if os.environ.get("REFILL"):  # take the freed range again (held) before the next engine
        q = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(q), ctypes.c_size_t(20 << 30)) == 0
        print(json.dumps({"phase": "a second 20 GB allocation held", "fps": rate()}), flush=True)
        assert hip.hipFree(q) == 0
    for mb in (int(x) for x in os.environ.get("HOSTPIN_MB", "").split(",") if x):
        b = pinned_empty((mb << 20,), np.uint8)
        b[::4096] = 1
        del b
        print(json.dumps({"phase": "after %d MB page-locked host alloc + free" % mb, "fps": rate()}), flush=True)
big_host()
print(json.dumps({"phase": "after 6.8 GB page-locked host", "fps": rate()}), flush=True)
big_engine()
print(json.dumps({"phase": "after a max_batch-384 engine", "fps": rate(), "device_cache": cache()}), flush=True)
print(json.dumps({"phase": "again", "fps": rate()}), flush=True)
print(json.dumps({"phase": "decisions only", "fps": rate(dec=True), "device_cache": cache()}), flush=True)
if os.environ.get("DEVICE"):  # device-API search time of the same frame (torch)
    import torch
    d = torch.from_numpy(synth_frames(W, H, 1, 0x1080, 0).astype(np.int16)).cuda()
    with MipEngine(W, H, max_batch=1) as eng:
        c = torch.empty((1, eng.costs_per_frame), dtype=torch.int32, device="cuda")
        eng.search_device(d, costs=c)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            eng.search_device(d, costs=c)
        torch.cuda.synchronize()
        print(json.dumps({"phase": "device API, 50 one-frame searches", "ms_each": round((time.perf_counter() - t0) / 50 * 1e3, 4)}), flush=True)
        hc = pinned_empty((1, eng.costs_per_frame), np.int32)
        t0 = time.perf_counter()
        for _ in range(20):
            eng.search(fr1, out={"cost": hc})
        print(json.dumps({"phase": "20 synchronous one-frame full calls", "ms_each": round((time.perf_counter() - t0) / 20 * 1e3, 4)}), flush=True)
