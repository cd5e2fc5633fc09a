"""ctypes binding of the C oracle (oracle/_ref/liboracle.so) -- test infrastructure only."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(REPO, "oracle", "_ref", "liboracle.so")

FILTERS = [
    "filterFrame_1d_int", "filterFrame_1d_float", "filterFrame_2d_int_quarterCtu",
    "filterFrame_2d_float_quarterCtu", "filterFrame_1d_int_5x5", "filterFrame_1d_float_5x5",
    "filterFrame_2d_int_5x5_quarterCtu", "filterFrame_2d_float_5x5_quarterCtu",
]

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
        L = ctypes.CDLL(LIB_PATH)
        u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
        i32p = ctypes.c_void_p
        L.mipo_search_ctus.argtypes = [u16p, u16p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       i32p, i32p, i32p, ctypes.c_int]
        L.mipo_filter_frame.argtypes = [u16p, u16p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.mipo_filter_frame.restype = ctypes.c_int
        L.mipo_synth_frame.argtypes = [u16p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
        L.mipo_num_ctus.argtypes = [ctypes.c_int, ctypes.c_int]
        L.mipo_num_ctus.restype = ctypes.c_int
        L.mipo_clip_counts.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def search(orig, refs=None, ctus=None, want_sad_satd=False, nthreads=0):
    """Oracle MIP search; returns cost (and sad, satd) int32 arrays of the whole frame
    (entries of CTUs outside `ctus` are left at 0)."""
    orig = np.ascontiguousarray(orig, np.uint16)
    refs = orig if refs is None else np.ascontiguousarray(refs, np.uint16)
    h, w = orig.shape
    n = lib().mipo_num_ctus(w, h)
    c0, c1 = (0, n) if ctus is None else ctus
    cost = np.zeros(n * 97840, np.int32)
    sad = np.zeros_like(cost) if want_sad_satd else None
    satd = np.zeros_like(cost) if want_sad_satd else None
    lib().mipo_search_ctus(orig, refs, w, h, c0, c1, _ptr(cost), _ptr(sad), _ptr(satd), nthreads)
    return (cost, sad, satd) if want_sad_satd else cost


def clip_counts(reset=True):
    """(below 0, above 1023) clip events of the oracle's reduced predictions since the last reset."""
    out = np.zeros(2, np.int64)
    lib().mipo_clip_counts(out.ctypes.data_as(ctypes.c_void_p), int(reset))
    return int(out[0]), int(out[1])


def filter_frame(frame, filter_name, kernel_idx):
    frame = np.ascontiguousarray(frame, np.uint16)
    out = np.zeros_like(frame)
    rc = lib().mipo_filter_frame(frame, out, frame.shape[1], frame.shape[0], FILTERS.index(filter_name), kernel_idx)
    if rc != 0:
        raise ValueError(f"oracle filter {filter_name}/{kernel_idx} unsupported (rc={rc})")
    return out


def synth(width, height, seed, kind=0):
    out = np.zeros((height, width), np.uint16)
    lib().mipo_synth_frame(out, width, height, seed, kind)
    return out
