#!/usr/bin/env python3
"""Host-buffer pipeline probe: end-to-end rates of mip_search_frames_async / mip_wait for
given call shapes (run under rocprofv3 --kernel-trace --memory-copy-trace to see the overlap
of H2D, filter, search and D2H; tools/trace_timeline.py summarises such a trace).

    python tools/e2e_probe.py [--calls 8] [--reps 3] CASE [CASE ...]

    python tools/e2e_probe.py --sync ... (synchronous calls one after the other)

CASE = FRAMES:OUT:HOST[:FILTER:KIDX][:mb=MAX_BATCH]
  FRAMES  frames per call (1080p unless --width/--height)
  OUT     dec (per-CU best mode + cost only) | full (int32 cost table)
  HOST    pinned (mip_host_alloc buffers) | pageable (malloc'd numpy arrays)
  FILTER  reference filter name (alternative references, engine filter), KIDX its KernelIdx
  mb=M    engine max_batch (default FRAMES: the drop-in's per-call engine, as bench.py's
          config sweep creates it)
Each case: an engine, one warm-up call, then `reps` rounds of `calls` asynchronous calls
queued back to back and one wait for the last; prints one JSON line per case (median rate,
all rates).  Cases are separated by 0.2 s of idle time (trace segments)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
import numpy as np  # noqa: E402

from mipgpu import MipEngine, pinned_empty  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402


def parse(case):
    parts = case.split(":")
    mb = None
    if parts[-1].startswith("mb="):
        mb = int(parts.pop()[3:])
    f, out, host = int(parts[0]), parts[1], parts[2]
    flt = parts[3] if len(parts) > 3 else None
    kidx = int(parts[4]) if len(parts) > 4 else 0
    assert out in ("dec", "full") and host in ("pinned", "pageable"), case
    return f, out, host, flt, kidx, mb or f


def torch_steps(step, W, H):
    """Use the GPU through torch as bench.py does, up to `step`: init | alloc | stream | d2h |
    d2h_pinned (each includes the ones before it, d2h_pinned excepted d2h)."""
    import torch
    steps = ["init", "alloc", "stream", "d2h", "d2h_pinned"]
    upto = steps.index(step)
    torch.cuda.set_device(0)
    torch.cuda.init()
    x = None
    if upto >= 1:
        x = torch.randint(0, 1024, (8, H, W), dtype=torch.int16, device="cuda")
    if upto >= 2:
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            x = x * 2
        torch.cuda.synchronize()
    if upto == 3:
        _ = x[:2].cpu()
    if upto == 4:
        h = torch.empty(x[:2].shape, dtype=x.dtype, pin_memory=True)
        h.copy_(x[:2], non_blocking=True)
    torch.cuda.synchronize()


def hip_runtimes():
    """The HIP runtime libraries mapped into this process (torch's wheel bundles its own;
    whichever is loaded first serves the engine)."""
    return sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln})


def run(case, W, H, calls, reps, torch_after=None, device_first=0, sync=False):
    F, out, host, flt, kidx, mb = parse(case)
    src = synth_frames(W, H, min(F, 4), 0x1080, 0)
    alloc = (lambda shape, dt: pinned_empty(shape, dt)) if host == "pinned" else (lambda shape, dt: np.zeros(shape, dt))
    frames = alloc((F, H, W), np.uint16)
    for i in range(F):
        frames[i] = src[i % src.shape[0]]
    with MipEngine(W, H, max_batch=mb, filter=flt, kernel_idx=kidx) as eng:
        if torch_after:  # torch's streams created after the engine's
            torch_steps(torch_after, W, H)
        if device_first:  # device-API searches of the same engine first (bench.py's timed steps)
            import torch
            d = torch.from_numpy(np.ascontiguousarray(frames).view(np.int16)).cuda()
            st = torch.cuda.Stream()
            for _ in range(device_first):
                eng.search_device(d, stream=st)
            torch.cuda.synchronize()
        if out == "dec":
            o = {"best_mode": alloc((F, eng.cus_per_frame), np.uint8), "best_cost": alloc((F, eng.cus_per_frame), np.int32)}
            kw = dict(costs=False, best=True, out=o)
        else:
            o = {"cost": alloc((F, eng.costs_per_frame), np.int32)}
            kw = dict(out=o)
        eng.search(frames, **kw)
        rates, enq, wt, call_us = [], [], [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            if sync:  # synchronous calls one after the other (mip_search_frames)
                for _ in range(calls):
                    eng.search(frames, **kw)
                tickets = []
                t1 = t2 = time.perf_counter()
            else:
                tickets, tc = [], [t0]
                for _ in range(calls):
                    tickets.append(eng.search_async(frames, **kw))
                    tc.append(time.perf_counter())
                call_us = [round(1e6 * (b - a), 1) for a, b in zip(tc, tc[1:])]
                t1 = time.perf_counter()
                eng.wait(tickets[-1])
                t2 = time.perf_counter()
            rates.append(calls * F / (t2 - t0))
            enq.append(1e3 * (t1 - t0))
            wt.append(1e3 * (t2 - t1))
            del tickets
        stats = eng.host_stats() if hasattr(eng, "host_stats") else None
    return {"case": case, "hip_runtime": hip_runtimes(), "frames_per_call": F, "out": out, "host": host, "filter": flt, "kernel_idx": kidx,
            "max_batch": mb, "calls": calls, "sync": sync, "fps": round(float(np.median(rates)), 1),
            "fps_all": [round(r, 1) for r in rates], "enqueue_ms": [round(x, 3) for x in enq],
            "wait_ms": [round(x, 3) for x in wt], "host_stats": stats, "last_round_call_us": call_us}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("cases", nargs="+")
    ap.add_argument("--calls", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--torch", default="", help="torch_steps(STEP) before the engines are created")
    ap.add_argument("--torch-after", default="", help="torch_steps(STEP) after each engine is created")
    ap.add_argument("--sync", action="store_true", help="synchronous calls (mip_search_frames) instead of queued ones")
    ap.add_argument("--device-first", type=int, default=0, help="device-API searches of the engine first")
    a = ap.parse_args()
    if a.torch:
        torch_steps(a.torch, a.width, a.height)
    for c in a.cases:
        print(json.dumps(run(c, a.width, a.height, a.calls, a.reps, a.torch_after, a.device_first, a.sync)), flush=True)
        time.sleep(0.2)


if __name__ == "__main__":
    main()
