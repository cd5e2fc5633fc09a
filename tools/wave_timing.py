#!/usr/bin/env python3
"""Per-task timing of the search kernel (MIPGPU_WAVE_TIMING instrumentation).

Runs one warm-up and one instrumented 1080p batch.  Reports, per size class, the mean wall
cycles of its tasks (under the kernel's normal co-residency) and per (task, mode pair) --
the data the host's task cost model (mipgpu.cpp pair_cost) is checked against -- and the
workgroup's summed task cycles per quadrant."""
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
path = os.path.join(tempfile.mkdtemp(), "clk.bin")
os.environ["MIPGPU_WAVE_TIMING"] = path
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mipgpu import MipEngine  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402

CLASSES = ["64x64", "32x32", "32x16", "16x32", "32x8", "8x32", "16x16", "16x8", "8x16", "32x4", "4x32",
           "16x4", "4x16", "8x8", "8x4", "4x8", "4x4", "32x8v2", "16x16v4", "16x8v2", "8x16v4"]
W, H, B, SLOTS = 1920, 1080, 8, 128
frames = torch.from_numpy(synth_frames(W, H, B, 0x1080, 0).astype(np.int16)).cuda()
eng = MipEngine(W, H, max_batch=B)
costs = torch.empty((B, eng.costs_per_frame), dtype=torch.int32, device="cuda")
eng.search_device(frames, costs=costs)
torch.cuda.synchronize()
os.remove(path)
eng.search_device(frames, costs=costs)
torch.cuda.synchronize()
tl = json.load(open(path + ".tasks"))
slices, lb, tasks = tl["slices"], tl["list_begin"], tl["tasks"]
# items are (frame, CTU, quadrant, slice); complete CTUs only (variant-0 lists)
clk = np.fromfile(path, dtype=np.uint64).astype(np.int64).reshape(B, eng.nctus, 4, slices, SLOTS)
full = [c for c in range(eng.nctus) if 128 * (c % (W // 128 + (W % 128 > 0)) + 1) <= W and 128 * (c // (W // 128 + (W % 128 > 0)) + 1) <= H]
mean_clk = clk[:, full].mean(axis=(0, 1))               # [quad, slice, task]
rows = {}
for q in range(4):
    for sl in range(slices):
        li = q * slices + sl
        for k, t in enumerate(range(lb[li], lb[li + 1])):
            cls, ncu, q0, q1 = tasks[t]
            rows.setdefault(cls, []).append((q1 - q0, ncu, mean_clk[q, sl, k]))
fit = {}
for cls, r in sorted(rows.items()):
    a = np.array(r, dtype=float)
    fit[CLASSES[cls]] = {"tasks": len(a), "mean_ncu": round(float(a[:, 1].mean()), 2),
                         "cycles_per_task_pair": round(float(a[:, 2].sum() / a[:, 0].sum())),
                         "total_cycles": round(float(a[:, 2].sum()))}
res = {"task_cycles_per_quadrant": mean_clk.sum(axis=(1, 2)).round().tolist(), "class": fit}
print(json.dumps(res, indent=1))
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
