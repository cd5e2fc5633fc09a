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


def masked(table, width, height):
    t = np.array(table, dtype="<i4", copy=True).reshape(-1)
    t[~layout.available_mask(width, height)] = layout.UNAVAILABLE
    return t


def ctu_row(fx, frame, ctu):
    raw = zlib.decompress(base64.b64decode(fx["frames"][frame]["ctu_rows"][str(ctu)]))
    return np.frombuffer(raw, "<i4")
