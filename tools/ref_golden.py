#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE kernels (oracle/_ref/ref_runner).

Runs on a GPU box (the reference's OpenCL kernels, compiled from /root/reference/intra.cl
by `make -C oracle ref`, executed by the AMD OpenCL runtime on the MI355X).

Which outputs are defined is established by experiment, not assumed: every configuration
runs the reference four times, with every device buffer (frame slots and their padding,
filtered frames, scratch, cost tables) filled with 0, 1023, 0x155 and 0 again
(`ref_runner --fill`).  Entries that differ between the runs depend on memory the reference
never wrote for the frame, or on the order of two work-groups' stores (the last run repeats
the first fill).  The C oracle's model of the undefined entries (oracle_lib.defined_mask:
CUs below the frame, linear reads past the frame end, reference samples the filters leave
undefined) must cover every changed entry (`fill_check`), and the oracle must equal the
reference on every other entry (`oracle_check`).  For each configuration the fixture
records, from the reference's own outputs (first run), with undefined entries set to
0x7fffffff (filtered samples: 0xffff):
  * SHA-256 of the masked int32 cost table and its per-shape sums,
  * the complete cost rows of a few CTUs (zlib+base64),
  * SAD / SATD hashes when the MAX_PERFORMANCE_DIST=0 build is used,
  * SHA-256 of the filtered frame for the alternative-reference configurations.

usage: python3 tools/ref_golden.py OUT_DIR [config-name ...]
"""
import base64
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time
import zlib

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from mipgpu import layout  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402

CONFIGS = {
    # name: (W, H, frames, kind, seed, filter, kernel_idx, full_dist, ctu_rows)
    "small_structured": (256, 256, 1, 0, 0x100, None, 0, True, [0, 3]),
    "small_uniform_partial": (384, 264, 1, 1, 0x264, None, 0, True, [1, 7]),
    "small_alt_2d_int": (384, 256, 2, 0, 0x3A0, "filterFrame_2d_int_quarterCtu", 1, True, [0, 4]),
    "small_alt_2d_float5": (256, 200, 2, 0, 0x3A1, "filterFrame_2d_float_5x5_quarterCtu", 2, True, [0, 2]),
    "small_alt_2d_int5": (256, 232, 1, 1, 0x3A2, "filterFrame_2d_int_5x5_quarterCtu", 1, False, [1]),
    "small_alt_2d_float3": (384, 136, 1, 0, 0x3A3, "filterFrame_2d_float_quarterCtu", 3, False, [2]),
    "c2_1080p_orig": (1920, 1080, 1, 0, 0x1080, None, 0, False, [0, 16, 134]),
    "c3_1080p_alt_float5": (1920, 1080, 2, 0, 0x1081, "filterFrame_2d_float_5x5_quarterCtu", 2, False, [0, 70]),
    "c1_1080p_uniform": (1920, 1080, 1, 1, 0x1082, None, 0, False, [5]),
    "c5_2160p_alt_int": (3840, 2160, 1, 0, 0x2160, "filterFrame_2d_int_quarterCtu", 0, False, [0, 509]),
    # separable filters (frame buffers zeroed by ref_runner; <= 2 frames so that rows read
    # below a frame are zeros, see oracle/mip_oracle.c filter_1d_tile3)
    "small_sep_1d_int": (384, 256, 2, 0, 0x3B0, "filterFrame_1d_int", 1, True, [0, 4]),
    "small_sep_1d_float": (256, 200, 2, 0, 0x3B1, "filterFrame_1d_float", 4, False, [0, 2]),
    "small_sep_1d_int_k3": (256, 256, 1, 1, 0x3B4, "filterFrame_1d_int", 3, False, [1]),
    "small_sep_1d_int5": (384, 232, 1, 1, 0x3B2, "filterFrame_1d_int_5x5", 2, False, [1]),
    "small_sep_1d_float5": (256, 136, 2, 0, 0x3B3, "filterFrame_1d_float_5x5", 1, False, [2]),
    "small_sep_1d_int5_k0": (128, 104, 1, 0, 0x3B5, "filterFrame_1d_int_5x5", 0, False, [0]),
    "c3s_1080p_sep_float5": (1920, 1080, 1, 0, 0x1083, "filterFrame_1d_float_5x5", 2, False, [0, 70]),
    "c3s_1080p_sep_int": (1920, 1080, 1, 0, 0x1084, "filterFrame_1d_int", 2, False, [16]),
    # float filters with scales whose fp32 quotient ties depend on the reference's division
    "small_alt_2d_float3_k2": (384, 256, 1, 0, 0x3A6, "filterFrame_2d_float_quarterCtu", 2, False, [0, 4]),
    "small_alt_2d_float3_k4": (256, 264, 1, 1, 0x3A7, "filterFrame_2d_float_quarterCtu", 4, False, [1]),
    # near-black frames: quotients around 1/2, where the reference's fp32 division decides
    "small_dark_2d_float3_k2": (256, 136, 1, 2, 0x3D0, "filterFrame_2d_float_quarterCtu", 2, False, [0]),
    "small_dark_2d_float3_k0": (256, 136, 1, 2, 0x3D1, "filterFrame_2d_float_quarterCtu", 0, False, [0]),
    "small_dark_1d_float_k4": (256, 136, 1, 2, 0x3D2, "filterFrame_1d_float", 4, False, [0]),
    "small_dark_2d_float5_k1": (256, 136, 1, 2, 0x3D3, "filterFrame_2d_float_5x5_quarterCtu", 1, False, [0]),
    "small_dark_1d_float5_k1": (256, 136, 1, 2, 0x3D4, "filterFrame_1d_float_5x5", 1, False, [0]),
    # the reference's own resolutions whose width is not a multiple of 128 (constants.h:17-23):
    # CUs right of the frame read the next row (linear indexes), the filters' last tile column
    # stores its wrapped columns over the next row (racing stores)
    "w416_orig": (416, 240, 2, 0, 0x416, None, 0, True, [3, 7]),
    "w416_2d_int": (416, 240, 2, 0, 0x417, "filterFrame_2d_int_quarterCtu", 1, True, [3, 7]),
    "w416_2d_float5": (416, 240, 1, 0, 0x41A, "filterFrame_2d_float_5x5_quarterCtu", 2, False, [3]),
    "w416_1d_int": (416, 240, 1, 0, 0x41B, "filterFrame_1d_int", 1, False, [7]),
    "w416_1d_float5": (416, 240, 1, 0, 0x41E, "filterFrame_1d_float_5x5", 1, False, [3]),
    "w416_2d_float": (416, 240, 1, 1, 0x418, "filterFrame_2d_float_quarterCtu", 2, False, [7]),
    "w416_2d_int5": (416, 240, 1, 1, 0x419, "filterFrame_2d_int_5x5_quarterCtu", 1, False, [3]),
    "w416_1d_float": (416, 240, 1, 1, 0x41C, "filterFrame_1d_float", 4, False, [7]),
    "w416_1d_int5": (416, 240, 1, 1, 0x41D, "filterFrame_1d_int_5x5", 2, False, [3]),
    "w832_orig": (832, 480, 1, 0, 0x832, None, 0, True, [6, 27]),
    "w832_2d_float5": (832, 480, 1, 0, 0x835, "filterFrame_2d_float_5x5_quarterCtu", 2, False, [13]),
    "w832_1d_int": (832, 480, 1, 0, 0x834, "filterFrame_1d_int", 2, False, [27]),
    "w1280_orig": (1280, 720, 1, 0, 0x1280, None, 0, False, [9, 59]),
    "w1280_2d_int": (1280, 720, 1, 0, 0x1283, "filterFrame_2d_int_quarterCtu", 0, False, [59]),
    "w1280_1d_float5": (1280, 720, 1, 0, 0x1282, "filterFrame_1d_float_5x5", 2, False, [29]),
    # BASELINE configs[3] geometry: 3840x2160 with original references
    "c4_2160p_orig": (3840, 2160, 1, 0, 0x2161, None, 0, False, [29, 509]),
}
FILLS = [0, 1023, 0x155, 0]  # the last run repeats the first fill: differences are races


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def pack_rows(costs, ctus):
    out = {}
    for c in ctus:
        row = np.ascontiguousarray(costs[c * layout.COSTS_PER_CTU:(c + 1) * layout.COSTS_PER_CTU], "<i4")
        out[str(c)] = base64.b64encode(zlib.compress(row.tobytes(), 9)).decode()
    return out


def masked(table, mask, fill=layout.UNAVAILABLE):
    t = table.copy()
    t[~mask] = fill
    return t


def summarize(costs, sad, satd, filt, masks, fundef, w, h, frames, rows):
    n = layout.num_ctus(w, h)
    per = n * layout.COSTS_PER_CTU
    res = {"frames": []}
    e = layout.ctu_entries()
    shape_of = np.tile(e["shape"], n)
    for f in range(frames):
        mask = masks[f]
        c = masked(costs[f * per:(f + 1) * per], mask)
        sums = np.bincount(shape_of[mask], weights=c[mask].astype(np.float64), minlength=47)
        fr = {"cost_sha256": sha(c), "shape_sums": [int(v) for v in sums], "defined_entries": int(mask.sum()),
              "ctu_rows": pack_rows(c, rows)}
        if sad is not None:
            fr["sad_sha256"] = sha(masked(sad[f * per:(f + 1) * per], mask))
            fr["satd_sha256"] = sha(masked(satd[f * per:(f + 1) * per], mask))
        if filt is not None:
            fr["filtered_sha256"] = sha(masked(filt[f], ~fundef[f], 0xFFFF))
            fr["filtered_undefined"] = int(fundef[f].sum())
        res["frames"].append(fr)
    return res


def run_ref(name, td, fill, tag):
    w, h, frames, kind, seed, filt, kidx, full, rows = CONFIGS[name]
    cmd = [os.path.join(REPO, "oracle", "_ref", "ref_runner"), "--bins", os.path.join(REPO, "oracle", "_ref"),
           "--width", str(w), "--height", str(h), "--frames", str(frames), "--synth", "%d:%x" % (kind, seed),
           "--fill", str(fill), "--out-cost", os.path.join(td, tag + "cost.i32")]
    if full:
        cmd += ["--full-dist", "--out-sad", os.path.join(td, tag + "sad.i32"), "--out-satd", os.path.join(td, tag + "satd.i32")]
    if filt:
        cmd += ["--filter", filt, "--kernel-idx", str(kidx), "--out-filtered", os.path.join(td, tag + "filt.u16")]
    line = subprocess.check_output(cmd, timeout=600).decode().strip().splitlines()[-1]
    costs = np.fromfile(os.path.join(td, tag + "cost.i32"), "<i4")
    sad = np.fromfile(os.path.join(td, tag + "sad.i32"), "<i4") if full else None
    satd = np.fromfile(os.path.join(td, tag + "satd.i32"), "<i4") if full else None
    fl = np.fromfile(os.path.join(td, tag + "filt.u16"), "<u2").reshape(frames, h, w) if filt else None
    return line, costs, sad, satd, fl


def run_config(name, out_dir):
    import oracle_lib as O
    w, h, frames, kind, seed, filt, kidx, full, rows = CONFIGS[name]
    n = layout.num_ctus(w, h)
    per = n * layout.COSTS_PER_CTU
    t0 = time.time()
    with tempfile.TemporaryDirectory() as td:
        runs = [run_ref(name, td, fill, "r%d_" % i) for i, fill in enumerate(FILLS)]
    t_ref = time.time() - t0
    line, costs, sad, satd, fl = runs[0]
    changed = np.zeros(costs.shape, bool)
    for r in runs[1:]:
        changed |= r[1] != costs
        if full:
            changed |= (r[2] != sad) | (r[3] != satd)
    fchanged = None
    if filt:
        fchanged = np.zeros(fl.shape, bool)
        for r in runs[1:]:
            fchanged |= r[4] != fl
    frames_in = synth_frames(w, h, frames, seed, kind)
    masks, fundef, checks, fills = [], [], [], []
    for f in range(frames):
        refs, und = O.filter_frame(frames_in[f], filt, kidx, with_undefined=True) if filt else (None, None)
        mask = O.defined_mask(w, h, und)
        masks.append(mask)
        fundef.append(und)
        oc, osad, osatd = O.search(frames_in[f], refs, want_sad_satd=True)
        rc = costs[f * per:(f + 1) * per]
        ch = changed[f * per:(f + 1) * per]
        ck = {"frame": f, "cost_mismatches": int(((oc != rc) & mask).sum())}
        fc = {"frame": f, "changed_entries": int(ch.sum()), "changed_but_defined_mismatches": int((ch & mask).sum()),
              "undefined_entries": int((~mask).sum())}
        if full:
            ck["sad_mismatches"] = int(((osad != sad[f * per:(f + 1) * per]) & mask).sum())
            ck["satd_mismatches"] = int(((osatd != satd[f * per:(f + 1) * per]) & mask).sum())
        if filt:
            ck["filtered_mismatches"] = int(((refs != fl[f]) & ~und).sum())
            fc["filtered_changed"] = int(fchanged[f].sum())
            fc["filtered_changed_but_defined_mismatches"] = int((fchanged[f] & ~und).sum())
            fc["filtered_undefined"] = int(und.sum())
        d = (oc != rc) & mask
        if d.any():
            idx = np.nonzero(d)[0][:5]
            ck["first_mismatch_idx"] = [int(i) for i in idx]
            ck["first_mismatch_ref_oracle"] = [[int(rc[i]), int(oc[i])] for i in idx]
        checks.append(ck)
        fills.append(fc)
    res = {"name": name, "format": 2,
           "config": {"width": w, "height": h, "frames": frames, "kind": kind, "seed": seed,
                      "filter": filt, "kernel_idx": kidx},
           "generator": "reference intra.cl kernels (oracle/_ref, AMD OpenCL) on GPU",
           "mask": "entries the reference defines: oracle_lib.defined_mask (fill experiment: fill_check)",
           "fills": FILLS, "ref_runner": json.loads(line), "ref_wall_s": t_ref}
    res.update(summarize(costs, sad, satd, fl, masks, fundef, w, h, frames, rows))
    res["oracle_check"] = checks
    res["fill_check"] = fills
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, name + ".json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(name, json.dumps(checks), json.dumps(fills), "ref %.1fs" % t_ref, flush=True)


if __name__ == "__main__":
    out = sys.argv[1]
    names = sys.argv[2:] or list(CONFIGS)
    for nm in names:
        run_config(nm, out)
