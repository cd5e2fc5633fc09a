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
per_item = clk.sum(axis=1) / 8.0  # 8 waves share an item's tasks
# placement: HW_ID cu_id bits 11:8, sh 12, se 15:13; XCC_ID low 4 bits of the high word
cu = ((hw >> 8) & 15) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | (((hw >> 32) & 15) << 8)
t0 = t0 - t0.min()
dur_us = (t1 - raw[:, SLOTS - 3].astype(np.int64)) / 100.0  # s_memrealtime: 100 MHz
ne = per_item > 0
print(json.dumps({"launch_span_us": float((t1.max() - raw[:, SLOTS - 3].astype(np.int64).min()) / 100.0),
                  "item_us_p50_p90_max": [round(float(np.percentile(dur_us[ne], p)), 1) for p in (50, 90, 100)],
                  "start_us_max": float(t0.max() / 100.0), "distinct_cus": int(len(set(cu.tolist()))),
                  "items_per_cu_max": int(np.bincount(np.unique(cu, return_inverse=True)[1]).max())}))
order = np.argsort(-dur_us)[:8]
print(json.dumps([{"item": int(i), "us": round(float(dur_us[i]), 1), "start_us": round(float(t0[i] / 100.0), 1),
                   "cu": int(cu[i])} for i in order]))
busy = per_item[per_item > 0]
q = np.percentile(busy, [50, 90, 99, 100])
print(json.dumps({"items": int(n), "nonempty": int(busy.size), "mean_cycles_per_wave": round(float(busy.mean())),
                  "p50": round(q[0]), "p90": round(q[1]), "p99": round(q[2]), "max": round(q[3]),
                  "max_over_mean": round(float(q[3] / busy.mean()), 3),
                  "tasks_per_item_max": int((clk > 0).sum(axis=1).max()),
                  "max_task_cycles": int(clk.max()), "sorted_top": sorted(busy.round().astype(int).tolist())[-12:]}))
