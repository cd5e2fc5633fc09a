#!/usr/bin/env python3
"""Time the fused search per CU-size class (MIPGPU_SHAPE_FILTER) on 1080p frames.

MIPGPU_SHAPE_FILTER is a profiling knob honoured only by a profiling build
(tools/build_variant.sh tools/bin/libmipgpu_prof.so -DMIPGPU_PROFILING_KNOBS); this script
loads that build (MIPGPU_LIB) -- the release library refuses the knob."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MIPGPU_LIB", os.path.join(REPO, "tools", "bin", "libmipgpu_prof.so"))
if not os.path.exists(os.environ["MIPGPU_LIB"]):
    sys.exit("%s missing: build it with tools/build_variant.sh tools/bin/libmipgpu_prof.so -DMIPGPU_PROFILING_KNOBS"
             % os.environ["MIPGPU_LIB"])
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mipgpu import MipEngine, layout  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402

W, H, B = 1920, 1080, 8
PMC = os.environ.get("SHAPE_PROFILE_PMC") == "1"  # 2 dispatches per class, in class order
frames = torch.from_numpy(synth_frames(W, H, B, 0x1080, 0).astype(np.int16)).cuda()
classes = {}
for s in layout.SHAPES:
    classes.setdefault((s.w, s.h), []).append(s.index)
res = {}
for (w, h), idx in sorted(classes.items(), key=lambda kv: -kv[0][0] * kv[0][1]):
    os.environ["MIPGPU_SHAPE_FILTER"] = ",".join(map(str, idx))
    eng = MipEngine(W, H, max_batch=B)
    costs = torch.empty((B, eng.costs_per_frame), dtype=torch.int32, device="cuda")
    eng.time_search_device(frames, costs, reps=1 if PMC else 2)
    ms = eng.time_search_device(frames, costs, reps=1 if PMC else 5) / B
    sm = sum(layout.SHAPES[i].ncu * layout.SHAPES[i].total_modes * w * h for i in idx) * layout.num_ctus(W, H)
    res["%dx%d" % (w, h)] = {"shapes": idx, "us_per_frame": round(ms * 1000, 2),
                             "ns_per_ksample_mode": round(ms * 1e6 / (sm / 1000), 3)}
    print("%5s shapes=%-30s %8.2f us/frame  %.3f ns per 1k sample-modes" % (
        "%dx%d" % (w, h), idx, ms * 1000, ms * 1e6 / (sm / 1000)), flush=True)
    eng.close()
os.environ.pop("MIPGPU_SHAPE_FILTER")
eng = MipEngine(W, H, max_batch=B)
costs = torch.empty((B, eng.costs_per_frame), dtype=torch.int32, device="cuda")
eng.time_search_device(frames, costs, reps=2)
tot = eng.time_search_device(frames, costs, reps=5) / B
print("all shapes: %.2f us/frame; sum of classes %.2f" % (tot * 1000, sum(v["us_per_frame"] for v in res.values())))
json.dump(res, open(sys.argv[1] if len(sys.argv) > 1 else "/dev/null", "w"), indent=1)
