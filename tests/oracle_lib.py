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
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        L.mipo_filter_frame_ex.argtypes = [u16p, u16p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.mipo_filter_frame_ex.restype = ctypes.c_int
        L.mipo_ref_undefined_cus.argtypes = [u8p, ctypes.c_int, ctypes.c_int, u8p]
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


def filter_frame(frame, filter_name, kernel_idx, with_undefined=False):
    """Oracle filter.  with_undefined: also return the bool mask of samples the reference
    leaves undefined (reads past the frame end, racing stores; mipo_filter_frame_ex)."""
    frame = np.ascontiguousarray(frame, np.uint16)
    out = np.zeros_like(frame)
    und = np.zeros(frame.shape, np.uint8)
    rc = lib().mipo_filter_frame_ex(frame, out, und, frame.shape[1], frame.shape[0], FILTERS.index(filter_name),
                                    kernel_idx)
    if rc != 0:
        raise ValueError(f"oracle filter {filter_name}/{kernel_idx} unsupported (rc={rc})")
    return (out, und.astype(bool)) if with_undefined else out


def defined_mask(width, height, refs_undefined=None):
    """Bool mask over a frame's cost table: entries the reference defines.  Geometric part:
    layout.available_mask (the engine's UNAVAILABLE set is its complement); with a filtered
    reference frame, also the CUs none of whose reference samples is undefined."""
    from mipgpu import layout
    m = layout.available_mask(width, height)
    if refs_undefined is None or not refs_undefined.any():
        return m
    cu = np.zeros(layout.num_ctus(width, height) * layout.CUS_PER_CTU, np.uint8)
    lib().mipo_ref_undefined_cus(np.ascontiguousarray(refs_undefined, np.uint8), width, height, cu)
    return m & ~layout.expand_cu_mask(cu.astype(bool), layout.num_ctus(width, height))


def synth(width, height, seed, kind=0):
    out = np.zeros((height, width), np.uint16)
    lib().mipo_synth_frame(out, width, height, seed, kind)
    return out
