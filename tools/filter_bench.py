#!/usr/bin/env python3
"""Device time and HBM roofline fraction of each of the eight filters (1080p x 32 frames,
HIP events on the launch stream)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mipgpu import FILTERS, filter_device  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402

W, H, REPS = 1920, 1080, 20
B = int(os.environ.get("FB_FRAMES", 32))       # frames per launch
KIDX = int(os.environ.get("FB_KIDX", 0))       # KernelIdx of every filter
ONLY = os.environ.get("FB_ONLY")               # one filter name
frames = torch.from_numpy(synth_frames(W, H, B, 0x1080, 0).astype(np.int16)).cuda()
out = torch.empty_like(frames)
s = torch.cuda.Stream()
res = {}
for name in FILTERS:
    if ONLY and name != ONLY:
        continue
    for _ in range(3):
        filter_device(frames, out, name, KIDX, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(REPS):
        filter_device(frames, out, name, KIDX, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / REPS
    gbs = 4 * W * H * B / (ms * 1e-3) / 1e9
    res[name] = {"ms_per_launch": round(ms, 4), "GB/s": round(gbs, 1), "frac_of_8TB/s": round(gbs / 8000, 3)}
# Calibration: a plain device-to-device copy of the same bytes (torch, same stream) -- the
# practically reachable read+write bandwidth for this size.
for _ in range(3):
    with torch.cuda.stream(s):
        out.copy_(frames)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
with torch.cuda.stream(s):
    for _ in range(REPS):
        out.copy_(frames)
e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / REPS
copy = {"ms_per_launch": round(ms, 4), "GB/s": round(4 * W * H * B / (ms * 1e-3) / 1e9, 1)}
try:  # the library's streaming copy (16 B per lane, 4 loads in flight): bench.py's calibration
    from mipgpu import copy_device
    for _ in range(3):
        copy_device(frames, out, stream=s)
    e0.record(s)
    for _ in range(REPS):
        copy_device(frames, out, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / REPS
    copy = {"torch_copy": copy, "ms_per_launch": round(ms, 4), "GB/s": round(4 * W * H * B / (ms * 1e-3) / 1e9, 1),
            "kernel": "mip_copy_device"}
except ImportError:
    pass
for v in res.values():
    v["frac_of_copy"] = round(copy["ms_per_launch"] / v["ms_per_launch"], 3)
print(json.dumps({"workload": "%dx%d x %d frames, kernel_idx %d" % (W, H, B, KIDX), "filters": res,
                  "copy_calibration": copy}, indent=1))
