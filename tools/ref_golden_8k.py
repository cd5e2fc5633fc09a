#!/usr/bin/env python3
"""BASELINE configs[4] pinned to the REFERENCE kernels: an 8K (7680x4320) frame with
alternative references (filterFrame_2d_int_quarterCtu, KernelIdx 0), run through the
reference's own OpenCL kernels (oracle/_ref/ref_runner) as overlapping CTU-row crops.

The reference cannot search a whole 8K frame: its reduced-prediction index
ctuIdx * 2 231 296 is an int and overflows for ctuIdx >= 963 (intra.cl:519-537; 2040 CTUs
at 8K).  A 7680-wide crop of at most 16 CTU rows holds at most 960 CTUs and fits.  A CTU
row's costs depend on the original samples of its CTUs, on the filtered row above it and
on the filtered column left of each CU (initBoundaries, intra.cl:96-107, 232-243), and a
filtered sample depends on the original samples one row / column around it (3x3 filter,
intra.cl:2856-3040).  So every crop overlaps its neighbours by one CTU row at each inner
edge (the filter's gates at a crop edge then only touch the overlap rows) and only its
interior CTU rows are kept: the kept rows' costs and filtered samples equal the whole
frame's.  W = 7680 is a multiple of 128, so no linear-index wrap crosses a crop either.

Bands (CTU rows [start, end) of the crop, kept rows [keep0, keep1)):
    [0, 16) keep [0, 15);  [14, 30) keep [15, 29);  [28, 34) keep [29, 34)
(the last crop ends at the frame's bottom, 4320 = 33.75 CTU rows, so its undefined CUs --
below the frame -- are the whole frame's).

As tools/ref_golden.py, every crop runs with the device buffers filled with 0, 1023, 0x155
and 0 again (ref_runner --fill): entries of the kept rows that change are undefined, and
the C oracle's whole-frame model must cover them (fill_check) and equal the reference on
every other entry (oracle_check).  The fixture (format 2, tests/golden/c6_4320p_alt_int.json)
holds the SHA-256 of the stitched, masked whole-frame cost table, its per-shape sums, a few
complete CTU rows (one per band and both band seams), and the stitched filtered frame's
hash -- the same fields as every other fixture, so tests/test_gpu_parity.py checks the HIP
engine's whole 8K table against it.

Runs on a GPU box (the reference kernels run on the MI355X through the AMD OpenCL runtime).
usage: python3 tools/ref_golden_8k.py OUT_DIR"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
from mipgpu import layout  # noqa: E402
from mipgpu.synth import synth_frames  # noqa: E402
from ref_golden import FILLS, summarize  # noqa: E402

NAME = "c6_4320p_alt_int"
W, H, KIND, SEED = 7680, 4320, 1, 0x8E  # the frame of tests/test_gpu_parity.py test_8k_alt_int_whole_table
FILTER, KIDX = "filterFrame_2d_int_quarterCtu", 0
BANDS = [(0, 16, 0, 15), (14, 30, 15, 29), (28, 34, 29, 34)]  # CTU rows: crop [a, b), keep [k0, k1)
ROWS = [0, 14 * 60 + 59, 15 * 60, 28 * 60 + 7, 29 * 60 + 30, 33 * 60 + 59]  # sample CTUs: bands and seams
MAX_CTUS = 962  # the reference's int32 prediction index: ctuIdx * 2 231 296 < 2^31


def run_crop(td, band_frame, hb, fill, tag):
    cols = (W + 127) // 128
    assert cols * ((hb + 127) // 128) <= MAX_CTUS, hb
    inp = os.path.join(td, tag + "in.u16")
    band_frame.astype("<u2").tofile(inp)
    cmd = [os.path.join(REPO, "oracle", "_ref", "ref_runner"), "--bins", os.path.join(REPO, "oracle", "_ref"),
           "--width", str(W), "--height", str(hb), "--frames", "1", "--input", inp, "--fill", str(fill),
           "--filter", FILTER, "--kernel-idx", str(KIDX), "--out-cost", os.path.join(td, tag + "cost.i32"),
           "--out-filtered", os.path.join(td, tag + "filt.u16")]
    line = subprocess.check_output(cmd, timeout=900).decode().strip().splitlines()[-1]
    cost = np.fromfile(os.path.join(td, tag + "cost.i32"), "<i4")
    filt = np.fromfile(os.path.join(td, tag + "filt.u16"), "<u2").reshape(hb, W)
    for f in ("in.u16", "cost.i32", "filt.u16"):
        os.remove(os.path.join(td, tag + f))
    return json.loads(line), cost, filt


def main(out_dir):
    import oracle_lib as O
    cols, n = W // 128, layout.num_ctus(W, H)
    per_ctu = layout.COSTS_PER_CTU
    frame = synth_frames(W, H, 1, SEED, KIND)[0]
    costs = np.zeros(n * per_ctu, np.int32)
    changed = np.zeros(n * per_ctu, bool)
    filt = np.zeros((H, W), np.uint16)
    fchanged = np.zeros((H, W), bool)
    runner, t0 = [], time.time()
    with tempfile.TemporaryDirectory() as td:
        for a, b, k0, k1 in BANDS:
            y0, y1 = 128 * a, min(H, 128 * b)
            band = np.ascontiguousarray(frame[y0:y1])
            runs = [run_crop(td, band, y1 - y0, fill, "b%d_r%d_" % (a, i)) for i, fill in enumerate(FILLS)]
            line, bc, bf = runs[0]
            runner.append({"crop_ctu_rows": [a, b], "kept_ctu_rows": [k0, k1], "height": y1 - y0, "ref_runner": line})
            # kept CTU rows: crop CTU index (r - a) * cols + c -> frame CTU index r * cols + c
            src = slice((k0 - a) * cols * per_ctu, (k1 - a) * cols * per_ctu)
            dst = slice(k0 * cols * per_ctu, k1 * cols * per_ctu)
            costs[dst] = bc[src]
            for r in runs[1:]:
                changed[dst] |= r[1][src] != bc[src]
            ys0, ys1 = 128 * k0, min(H, 128 * k1)
            filt[ys0:ys1] = bf[ys0 - y0:ys1 - y0]
            for r in runs[1:]:
                fchanged[ys0:ys1] |= r[2][ys0 - y0:ys1 - y0] != bf[ys0 - y0:ys1 - y0]
            print("band %s done (%.0f s)" % ((a, b, k0, k1), time.time() - t0), flush=True)
    t_ref = time.time() - t0
    refs, und = O.filter_frame(frame, FILTER, KIDX, with_undefined=True)
    mask = O.defined_mask(W, H, und)
    oc = O.search(frame, refs)
    check = {"frame": 0, "cost_mismatches": int(((oc != costs) & mask).sum()),
             "filtered_mismatches": int(((refs != filt) & ~und).sum())}
    d = (oc != costs) & mask
    if d.any():
        idx = np.nonzero(d)[0][:5]
        check["first_mismatch_idx"] = [int(i) for i in idx]
        check["first_mismatch_ref_oracle"] = [[int(costs[i]), int(oc[i])] for i in idx]
    fill = {"frame": 0, "changed_entries": int(changed.sum()), "changed_but_defined_mismatches": int((changed & mask).sum()),
            "undefined_entries": int((~mask).sum()), "filtered_changed": int(fchanged.sum()),
            "filtered_changed_but_defined_mismatches": int((fchanged & ~und).sum()), "filtered_undefined": int(und.sum())}
    res = {"name": NAME, "format": 2,
           "config": {"width": W, "height": H, "frames": 1, "kind": KIND, "seed": SEED, "filter": FILTER,
                      "kernel_idx": KIDX},
           "generator": "reference intra.cl kernels (oracle/_ref, AMD OpenCL) on GPU, as 7680-wide crops of <= 16 CTU "
                        "rows (<= 960 CTUs: the reference's int32 prediction index, intra.cl:519-537) overlapping by "
                        "one CTU row at every inner edge; interior CTU rows and filtered rows stitched "
                        "(tools/ref_golden_8k.py)",
           "mask": "entries the reference defines: oracle_lib.defined_mask (fill experiment: fill_check)",
           "fills": FILLS, "crops": runner, "ref_wall_s": t_ref}
    res.update(summarize(costs, None, None, filt[None], [mask], [und], W, H, 1, ROWS))
    res["oracle_check"] = [check]
    res["fill_check"] = [fill]
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, NAME + ".json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(NAME, json.dumps(check), json.dumps(fill), "ref %.1fs" % t_ref, flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
