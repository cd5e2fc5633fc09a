#!/usr/bin/env python3
"""Per-item cost distribution of a small launch (MIPGPU_WAVE_TIMING instrumentation): one
1080p frame, one slice per quadrant; per item (quadrant) the summed task cycles of its
waves, against the host's cost model (pick_work / the LPT order).  GPU box."""
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

W, H, SLOTS = 1920, 1080, 128
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
frames = torch.from_numpy(synth_frames(W, H, B, 0x1080, 0).astype(np.int16)).cuda()
eng = MipEngine(W, H, max_batch=B, slices_per_ctu=1)
costs = torch.empty((B, eng.costs_per_frame), dtype=torch.int32, device="cuda")
eng.search_device(frames, costs=costs)
torch.cuda.synchronize()
os.remove(path)
eng.search_device(frames, costs=costs)
torch.cuda.synchronize()
raw = np.fromfile(path, dtype=np.uint64)
n = raw.size // SLOTS
raw = raw.reshape(n, SLOTS)
t0, t1, hw = raw[:, SLOTS - 3].astype(np.int64), raw[:, SLOTS - 2].astype(np.int64), raw[:, SLOTS - 1]
clk = raw[:, :SLOTS - 3].astype(np.int64)
per_item = clk.sum(axis=1)  # cycles of all the item's tasks (shader clock; 8 or 16 waves share them)
# placement: HW_ID cu_id bits 11:8, sh 12, se 15:13; XCC_ID low 4 bits of the high word
ne = per_item > 0
s0 = raw[:, SLOTS - 3].astype(np.int64)
t0 = s0[ne].min()
cu = ((hw >> 8) & 15) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | (((hw >> 32) & 15) << 8)
rows = np.stack([np.arange(n)[ne], (s0[ne] - t0), (t1[ne] - t0), cu[ne].astype(np.int64), per_item[ne].astype(np.int64)], 1)
out = os.environ.get("ITEM_CSV")
if out:
    np.savetxt(out, rows, fmt="%d", delimiter=",", header="item,start_10ns,end_10ns,cu,task_cycles_sum")
dur = (rows[:, 2] - rows[:, 1]) / 100.0
print(json.dumps({"launch_span_us": float(rows[:, 2].max() / 100.0), "last_start_us": float(rows[:, 1].max() / 100.0),
                  "item_us_p10_p50_p90_max": [round(float(np.percentile(dur, p)), 1) for p in (10, 50, 90, 100)],
                  "distinct_cus": int(len(set(rows[:, 3].tolist()))),
                  "max_items_per_cu": int(np.bincount(np.unique(rows[:, 3], return_inverse=True)[1]).max())}))
