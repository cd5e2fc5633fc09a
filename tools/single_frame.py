#!/usr/bin/env python3
"""Single-frame launches only (the per-frame encoder path): N one-frame 1080p searches back
to back on one stream, for a kernel trace of exactly that launch shape
(`rocprofv3 --kernel-trace --stats -- python3 tools/single_frame.py [N]`).  GPU box."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vvc-mip-gpu_amd"))
import torch  # noqa: E402

from mipgpu import MipEngine, build_id  # noqa: E402
from mipgpu.synth import synth_frames_torch  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda", 0)
frame = synth_frames_torch(1920, 1080, 1, 0x51F, 0, device=dev)
eng = MipEngine(1920, 1080)
costs = torch.empty((1, eng.costs_per_frame), dtype=torch.int32, device=dev)
s = torch.cuda.Stream(dev)
for _ in range(5):
    eng.search_device(frame, costs=costs, stream=s)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(N):
    eng.search_device(frame, costs=costs, stream=s)
e1.record(s)
torch.cuda.synchronize(dev)
print(json.dumps({"build_id": build_id(), "launches": N, "event_ms_per_launch": round(e0.elapsed_time(e1) / N, 4)}))
