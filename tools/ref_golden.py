#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE kernels (oracle/_ref/ref_runner).

Runs on a GPU box (the reference's OpenCL kernels, compiled from /root/reference/intra.cl
by `make -C oracle ref`, executed by the AMD OpenCL runtime on the MI355X).  For each
configuration it records, from the reference's own outputs:
  * SHA-256 of the masked int32 cost table (CUs not fully inside the frame -> 0x7fffffff,
    because the reference leaves them undefined: stale LDS, intra.cl:96-98 / 717),
  * per-shape sums of the masked costs,
  * the complete cost rows of a few CTUs (zlib+base64),
  * SAD / SATD hashes when the MAX_PERFORMANCE_DIST=0 build is used,
  * SHA-256 of the filtered frame for the alternative-reference configurations,
and, as a first cross-check, the same hashes computed by the C oracle on the host CPU.

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
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def pack_rows(costs, ctus):
    out = {}
    for c in ctus:
        row = np.ascontiguousarray(costs[c * layout.COSTS_PER_CTU:(c + 1) * layout.COSTS_PER_CTU], "<i4")
        out[str(c)] = base64.b64encode(zlib.compress(row.tobytes(), 9)).decode()
    return out


def masked(table, mask):
    t = table.copy()
    t[~mask] = layout.UNAVAILABLE
    return t


def summarize(costs, sad, satd, filt, w, h, frames, rows):
    n = layout.num_ctus(w, h)
    mask = layout.available_mask(w, h)
    per = n * layout.COSTS_PER_CTU
    res = {"frames": []}
    for f in range(frames):
        c = masked(costs[f * per:(f + 1) * per], mask)
        e = layout.ctu_entries()
        shape_of = np.tile(e["shape"], n)
        sums = np.bincount(shape_of[mask], weights=c[mask].astype(np.float64), minlength=47)
        fr = {"cost_sha256": sha(c), "shape_sums": [int(v) for v in sums],
              "ctu_rows": pack_rows(c, rows)}
        if sad is not None:
            fr["sad_sha256"] = sha(masked(sad[f * per:(f + 1) * per], mask))
            fr["satd_sha256"] = sha(masked(satd[f * per:(f + 1) * per], mask))
        if filt is not None:
            fr["filtered_sha256"] = sha(filt[f])
        res["frames"].append(fr)
    return res


def run_config(name, out_dir, with_oracle=True):
    w, h, frames, kind, seed, filt, kidx, full, rows = CONFIGS[name]
    n = layout.num_ctus(w, h)
    per = n * layout.COSTS_PER_CTU
    with tempfile.TemporaryDirectory() as td:
        cmd = [os.path.join(REPO, "oracle", "_ref", "ref_runner"), "--bins", os.path.join(REPO, "oracle", "_ref"),
               "--width", str(w), "--height", str(h), "--frames", str(frames), "--synth", "%d:%x" % (kind, seed),
               "--out-cost", os.path.join(td, "cost.i32")]
        if full:
            cmd += ["--full-dist", "--out-sad", os.path.join(td, "sad.i32"), "--out-satd", os.path.join(td, "satd.i32")]
        if filt:
            cmd += ["--filter", filt, "--kernel-idx", str(kidx), "--out-filtered", os.path.join(td, "filt.u16")]
        t0 = time.time()
        line = subprocess.check_output(cmd, timeout=600).decode().strip().splitlines()[-1]
        t_ref = time.time() - t0
        costs = np.fromfile(os.path.join(td, "cost.i32"), "<i4")
        sad = np.fromfile(os.path.join(td, "sad.i32"), "<i4") if full else None
        satd = np.fromfile(os.path.join(td, "satd.i32"), "<i4") if full else None
        fl = np.fromfile(os.path.join(td, "filt.u16"), "<u2").reshape(frames, h, w) if filt else None
    res = {"name": name, "config": {"width": w, "height": h, "frames": frames, "kind": kind, "seed": seed,
                                    "filter": filt, "kernel_idx": kidx},
           "generator": "reference intra.cl kernels (oracle/_ref, AMD OpenCL) on GPU",
           "ref_runner": json.loads(line), "ref_wall_s": t_ref}
    res.update(summarize(costs, sad, satd, fl, w, h, frames, rows))
    if with_oracle:
        import oracle_lib as O
        frames_in = synth_frames(w, h, frames, seed, kind)
        checks = []
        for f in range(frames):
            refs = O.filter_frame(frames_in[f], filt, kidx) if filt else None
            oc, osad, osatd = O.search(frames_in[f], refs, want_sad_satd=True)
            mask = layout.available_mask(w, h)
            rc = costs[f * per:(f + 1) * per]
            d = (oc != rc) & mask
            ck = {"frame": f, "cost_mismatches": int(d.sum())}
            if full:
                ck["sad_mismatches"] = int(((osad != sad[f * per:(f + 1) * per]) & mask).sum())
                ck["satd_mismatches"] = int(((osatd != satd[f * per:(f + 1) * per]) & mask).sum())
            if filt:
                ck["filtered_mismatches"] = int((refs != fl[f]).sum())
                ck["filtered_maxdiff"] = int(np.abs(refs.astype(int) - fl[f].astype(int)).max())
            if d.any():
                idx = np.nonzero(d)[0][:5]
                ck["first_mismatch_idx"] = [int(i) for i in idx]
                ck["first_mismatch_ref_oracle"] = [[int(rc[i]), int(oc[i])] for i in idx]
            checks.append(ck)
        res["oracle_check"] = checks
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, name + ".json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(name, json.dumps(res.get("oracle_check")), "ref %.1fs" % t_ref, flush=True)


if __name__ == "__main__":
    out = sys.argv[1]
    names = sys.argv[2:] or list(CONFIGS)
    for nm in names:
        run_config(nm, out)
