#!/usr/bin/env python3
"""Small-launch latency of the search (the per-frame encoder path, main.cpp:678-1241 searches
one frame per iteration): device time per launch of 1..N resident 1080p frames, for the
engine's automatic choice and for fixed slice counts, with the longest-first item order
(default) and, MIPGPU_ORDER=0, the raster order.  One JSON line per configuration.
usage: tools/small_batch.py [W H] (GPU box)"""
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vvc-mip-gpu_amd"))
import torch  # noqa: E402

from mipgpu import MipEngine, build_id  # noqa: E402
from mipgpu.synth import synth_frames_torch  # noqa: E402

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1920, 1080)
NF = [1, 2, 3, 4, 8, 16]
dev = torch.device("cuda", 0)
frames = synth_frames_torch(W, H, max(NF), 0x5B, 0, device=dev)
s = torch.cuda.Stream(dev)


# SB_DEC=1: decisions only (no cost table); SB_FILTER=NAME[:IDX]: the engine's alternative
# references (filter + search per launch)
DEC = os.environ.get("SB_DEC") == "1"
FILT = os.environ.get("SB_FILTER")


def run(eng, n, reps=40):
    if DEC:
        kw = dict(costs=False, best_mode=torch.empty((n, eng.cus_per_frame), dtype=torch.uint8, device=dev),
                  best_cost=torch.empty((n, eng.cus_per_frame), dtype=torch.int32, device=dev))
    else:
        kw = dict(costs=torch.empty((n, eng.costs_per_frame), dtype=torch.int32, device=dev))
    for _ in range(5):
        eng.search_device(frames[:n], stream=s, **kw)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        eng.search_device(frames[:n], stream=s, **kw)
    e1.record(s)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / reps


print(json.dumps({"build_id": build_id(), "size": [W, H]}), flush=True)
# SB_CUTS: task cut factors to try (MIPGPU_CUT_FACTOR, engine creation); SB_WIDE: 16-wave workgroups (MIPGPU_WIDE: 0 never, 1 every small launch, "auto"
# the engine's rule); SB_ORDERS: 1 = LPT, 0 = raster; SB_SLICES: 0 = the engine's choice
grid = itertools.product(os.environ.get("SB_CUTS", "2").split(","),
                         os.environ.get("SB_WIDE", "auto").split(","), os.environ.get("SB_ORDERS", "1,0").split(","),
                         map(int, os.environ.get("SB_SLICES", "0,1,2,4").split(",")))
for cut, wide, order, sl in grid:
    os.environ["MIPGPU_CUT_FACTOR"] = cut
    os.environ["MIPGPU_ORDER"] = order
    if wide == "auto":
        os.environ.pop("MIPGPU_WIDE", None)
    else:
        os.environ["MIPGPU_WIDE"] = wide
    fkw = {}
    if FILT:
        fkw = dict(filter=FILT.split(":")[0], kernel_idx=int(FILT.split(":")[1]) if ":" in FILT else 0)
    eng = MipEngine(W, H, max_batch=max(NF), slices_per_ctu=sl, **fkw)
    res = {n: round(run(eng, n), 4) for n in NF}
    eng.close()
    print(json.dumps({"cut": float(cut), "wide": wide, "dec": DEC, "filter": FILT, "order": "lpt" if order == "1" else "raster",
                      "slices": sl or "auto",
                      "ms_per_launch": res,
                      "frames_per_s": {n: round(n / (ms * 1e-3), 1) for n, ms in res.items()}}), flush=True)
