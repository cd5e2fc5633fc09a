#!/usr/bin/env python3
"""Do back-to-back small searches gain from overlapping?  N device-API searches of F resident
1080p frames each (`mip_search_device`), all on one stream vs alternating over S streams
(the next launch's workgroups can take CUs while the previous launch drains), decisions only
or full tables.  Prints one JSON line per case: frames/s (median of reps).

    python tools/overlap_probe.py [--frames 1] [--launches 200] [--reps 5] [--streams 1 2 3]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mipgpu import MipEngine  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1)
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--dec", action="store_true", help="decisions only (no cost table)")
    a = ap.parse_args()
    W, H, F = 1920, 1080, a.frames
    torch.cuda.init()
    fr = synth_frames(W, H, F, 0x77, 0)
    d = torch.from_numpy(fr.astype(np.int16)).cuda()
    with MipEngine(W, H, max_batch=F) as eng:
        n = eng.cus_per_frame
        outs = []
        for _ in range(max(a.streams)):
            if a.dec:
                outs.append(dict(costs=False, best_mode=torch.empty((F, n), dtype=torch.uint8, device="cuda"),
                                 best_cost=torch.empty((F, n), dtype=torch.int32, device="cuda")))
            else:
                outs.append(dict(costs=torch.empty((F, eng.costs_per_frame), dtype=torch.int32, device="cuda")))
        streams = [torch.cuda.Stream() for _ in range(max(a.streams))]
        for ns in a.streams:
            rates = []
            for rep in range(a.reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(a.launches):
                    eng.search_device(d, stream=streams[i % ns], **outs[i % ns])
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                if rep:
                    rates.append(a.launches * F / dt)
            print(json.dumps({"frames_per_launch": F, "streams": ns, "dec": a.dec, "launches": a.launches,
                              "fps": round(float(np.median(rates)), 1), "fps_all": [round(r, 1) for r in rates]}),
                  flush=True)


if __name__ == "__main__":
    main()
