#!/usr/bin/env python3
"""Latency of ONE large frame split into CTU-row bands over N GPUs:
every rank holds the whole frame (same seed), searches its band with
mip_search_device_range, the band tables are gathered and rank 0 checks the assembled
table against a whole-frame search.  One JSON line from rank 0.

    python tools/band_latency.py [--width 7680 --height 4320 --filter NAME --kernel-idx K]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/band_latency.py
(--backend gloo lets several ranks share one GPU for a functional run.)"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--filter", default="filterFrame_2d_int_quarterCtu")
    ap.add_argument("--kernel-idx", type=int, default=0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--backend", default="nccl")
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    from mipgpu import MipEngine
    from mipgpu.split import ctu_row_bands, gather_bands
    from mipgpu.synth import synth_frames

    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group(args.backend, **({"device_id": torch.device("cuda", local)}
                                                 if args.backend == "nccl" else {}))
    W, H = args.width, args.height
    frame = torch.from_numpy(synth_frames(W, H, 1, 0x4320, 0).astype(np.int16)).cuda()
    b, e = ctu_row_bands(W, H, world)[rank]
    with MipEngine(W, H, device=local, filter=args.filter, kernel_idx=args.kernel_idx) as eng:
        costs = torch.zeros((1, eng.costs_per_frame), dtype=torch.int32, device="cuda")
        for _ in range(2):
            eng.search_device_range(frame, b, e, costs)
        torch.cuda.synchronize()
        ms = []
        for _ in range(args.reps):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.search_device_range(frame, b, e, costs)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([dt], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                dt = float(t.item())
            ms.append(1000 * dt)
        full = gather_bands(costs.cpu().numpy(), W, H, rank, world) if world > 1 else costs.cpu().numpy()
        ok = None
        if rank == 0:
            ref = eng.search_device(frame).cpu().numpy()
            ok = bool(np.array_equal(full, ref))
    if rank == 0:
        print(json.dumps({"frame": "%dx%d" % (W, H), "filter": args.filter, "ranks": world, "band_ctus": e - b,
                          "ms_per_frame_median": round(float(np.median(ms)), 4), "assembled_equals_whole": ok}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
