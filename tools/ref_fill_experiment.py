#!/usr/bin/env python3
"""Which reference outputs are defined?  Runs the REFERENCE kernels (oracle/_ref/ref_runner)
on the same frames with different fill values in every device buffer (frame slots and their
padding, filtered frames, scratch, cost tables) and once more with the first fill (races).

An output entry that changes between runs depends on memory the reference did not write for
this frame -- reads past the end of the frame (linear indexes of the last CTU / tile column
wrap into the next row and, in the last row, past the frame), stale scratch, or a write race
between two workgroups (the filters' tiles at widths that are not multiples of 128 write
the wrapped part of their rows over their neighbours' samples).  Everything else is the
reference's deterministic output.

GPU box only.  usage: python3 tools/ref_fill_experiment.py OUT_DIR [config ...]
Writes OUT_DIR/<config>.json (counts) and, for configs marked `pull`, OUT_DIR/<config>.npz
(the first run's int32 cost table and filtered frame plus bit masks of the changed entries).
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILLS = [0, 1023, 0x155, 0]  # the last run repeats the first fill: differences are races

CONFIGS = {
    # name: (W, H, frames, kind, seed, filter, kernel_idx, pull)
    "w416_orig": (416, 240, 2, 0, 0x416, None, 0, True),
    "w416_2d_int": (416, 240, 2, 0, 0x417, "filterFrame_2d_int_quarterCtu", 1, True),
    "w416_2d_float": (416, 240, 1, 0, 0x418, "filterFrame_2d_float_quarterCtu", 2, True),
    "w416_2d_int5": (416, 240, 1, 1, 0x419, "filterFrame_2d_int_5x5_quarterCtu", 1, True),
    "w416_2d_float5": (416, 240, 2, 0, 0x41A, "filterFrame_2d_float_5x5_quarterCtu", 2, True),
    "w416_1d_int": (416, 240, 2, 0, 0x41B, "filterFrame_1d_int", 1, True),
    "w416_1d_float": (416, 240, 1, 0, 0x41C, "filterFrame_1d_float", 4, True),
    "w416_1d_int5": (416, 240, 1, 1, 0x41D, "filterFrame_1d_int_5x5", 2, True),
    "w416_1d_float5": (416, 240, 1, 0, 0x41E, "filterFrame_1d_float_5x5", 1, True),
    "w832_orig": (832, 480, 1, 0, 0x832, None, 0, True),
    "w832_2d_int": (832, 480, 1, 0, 0x833, "filterFrame_2d_int_quarterCtu", 0, True),
    "w832_1d_int": (832, 480, 1, 0, 0x834, "filterFrame_1d_int", 2, True),
    "w1280_orig": (1280, 720, 1, 0, 0x1280, None, 0, False),
    "w1280_2d_float5": (1280, 720, 1, 0, 0x1281, "filterFrame_2d_float_5x5_quarterCtu", 2, False),
    "w1280_1d_float5": (1280, 720, 1, 0, 0x1282, "filterFrame_1d_float_5x5", 2, False),
    "w1920_orig": (1920, 1080, 1, 0, 0x1080, None, 0, False),
    "w1920_1d_int": (1920, 1080, 1, 0, 0x1084, "filterFrame_1d_int", 2, False),
    "w3840_orig": (3840, 2160, 1, 0, 0x2161, None, 0, False),
}


def run(cfg, fill, td, tag):
    w, h, frames, kind, seed, filt, kidx, _ = cfg
    cmd = [os.path.join(REPO, "oracle", "_ref", "ref_runner"), "--bins", os.path.join(REPO, "oracle", "_ref"),
           "--width", str(w), "--height", str(h), "--frames", str(frames), "--synth", "%d:%x" % (kind, seed),
           "--fill", str(fill), "--out-cost", os.path.join(td, tag + ".i32")]
    if filt:
        cmd += ["--filter", filt, "--kernel-idx", str(kidx), "--out-filtered", os.path.join(td, tag + ".u16")]
    subprocess.check_output(cmd, timeout=600)
    cost = np.fromfile(os.path.join(td, tag + ".i32"), "<i4")
    fl = np.fromfile(os.path.join(td, tag + ".u16"), "<u2") if filt else None
    return cost, fl


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    names = sys.argv[2:] or list(CONFIGS)
    for name in names:
        cfg = CONFIGS[name]
        w, h, frames = cfg[0], cfg[1], cfg[2]
        t0 = time.time()
        with tempfile.TemporaryDirectory() as td:
            runs = [run(cfg, f, td, "r%d" % i) for i, f in enumerate(FILLS)]
        cost0, fl0 = runs[0]
        fill_changed = np.zeros(cost0.shape, bool)
        for c, _ in runs[1:-1]:
            fill_changed |= c != cost0
        race_changed = runs[-1][0] != cost0
        res = {"name": name, "width": w, "height": h, "frames": frames, "kind": cfg[3], "seed": cfg[4],
               "filter": cfg[5], "kernel_idx": cfg[6], "fills": FILLS,
               "cost_entries": int(cost0.size), "cost_changed_by_fill": int(fill_changed.sum()),
               "cost_changed_by_repeat": int(race_changed.sum()), "seconds": round(time.time() - t0, 1)}
        arrays = {"cost": cost0, "cost_fill_changed": np.packbits(fill_changed),
                  "cost_race_changed": np.packbits(race_changed)}
        if fl0 is not None:
            ffill = np.zeros(fl0.shape, bool)
            for _, f in runs[1:-1]:
                ffill |= f != fl0
            frace = runs[-1][1] != fl0
            res["filtered_changed_by_fill"] = int(ffill.sum())
            res["filtered_changed_by_repeat"] = int(frace.sum())
            arrays.update(filtered=fl0, filtered_fill_changed=np.packbits(ffill),
                          filtered_race_changed=np.packbits(frace))
            # positions (frame, y, x) of the first changed samples, for the record
            for key, m in (("filtered_fill_first", ffill), ("filtered_race_first", frace)):
                idx = np.nonzero(m)[0][:16]
                res[key] = [[int(i // (w * h)), int(i % (w * h) // w), int(i % w)] for i in idx]
        with open(os.path.join(out, name + ".json"), "w") as fh:
            json.dump(res, fh, indent=1)
        if cfg[7]:
            np.savez_compressed(os.path.join(out, name + ".npz"), **arrays)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
