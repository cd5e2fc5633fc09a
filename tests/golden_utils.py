"""Helpers for the golden fixtures in tests/golden/ (produced by tools/ref_golden.py from
the REFERENCE's own OpenCL kernels running on an MI355X; see tests/golden/README.md)."""
import base64
import glob
import hashlib
import json
import os
import zlib

import numpy as np

from mipgpu import layout
from mipgpu.synth import synth_frames

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.json")))


def load(name):
    with open(os.path.join(GOLDEN_DIR, name + ".json")) as f:
        return json.load(f)


def inputs(fx):
    c = fx["config"]
    return synth_frames(c["width"], c["height"], c["frames"], c["seed"], c["kind"])


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def refs_and_mask(fx, frames, f):
    """(filtered reference frame or None, its undefined-sample mask or None, defined-entry
    mask of the cost table) of frame f of a fixture, from the C oracle (the fixture's
    fill_check shows the oracle's undefined set covers every entry the reference left
    undefined in the fill experiment, see tools/ref_golden.py)."""
    import oracle_lib as O
    c = fx["config"]
    refs, und = (None, None)
    if c["filter"]:
        refs, und = O.filter_frame(frames[f], c["filter"], c["kernel_idx"], with_undefined=True)
    return refs, und, O.defined_mask(c["width"], c["height"], und)


def masked(table, mask, fill=layout.UNAVAILABLE):
    t = np.array(table, copy=True).reshape(-1)
    t[~np.asarray(mask).reshape(-1)] = fill
    return t


def filtered_sha(frame, undefined):
    return sha(masked(np.asarray(frame, "<u2"), ~undefined, 0xFFFF))


def ctu_row(fx, frame, ctu):
    raw = zlib.decompress(base64.b64decode(fx["frames"][frame]["ctu_rows"][str(ctu)]))
    return np.frombuffer(raw, "<i4")
