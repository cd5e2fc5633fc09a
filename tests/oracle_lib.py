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


def filter_frame(frame, filter_name, kernel_idx, with_undefined=False, kinds=False):
    """Oracle filter.  with_undefined: also return the bool mask of samples the reference
    leaves undefined (reads past the frame end, racing stores; mipo_filter_frame_ex); kinds:
    that mask as codes instead (bit 0 = poison: reads past the frame's end, bit 1 = a racing
    store with a different value)."""
    frame = np.ascontiguousarray(frame, np.uint16)
    out = np.zeros_like(frame)
    und = np.zeros(frame.shape, np.uint8)
    rc = lib().mipo_filter_frame_ex(frame, out, und, frame.shape[1], frame.shape[0], FILTERS.index(filter_name),
                                    kernel_idx)
    if rc != 0:
        raise ValueError(f"oracle filter {filter_name}/{kernel_idx} unsupported (rc={rc})")
    if not with_undefined:
        return out
    return out, (und if kinds else und.astype(bool))


def engine_unavailable_mask(frame, filter_name, kernel_idx):
    """Entries the engine reports MIP_COST_UNAVAILABLE when it filters the references itself:
    the geometrically undefined CUs and the CUs that read a filtered sample the reference's
    filter computes from memory past the frame's end (poison, bit 0 of the oracle's codes).
    CUs whose reference samples only race (bit 1) get the owning tile's value, one of the
    reference's outcomes."""
    from mipgpu import layout
    w, h = frame.shape[1], frame.shape[0]
    if filter_name is None:
        return ~layout.available_mask(w, h)
    _, und = filter_frame(frame, filter_name, kernel_idx, with_undefined=True, kinds=True)
    return ~defined_mask(w, h, (und & 1).astype(bool))


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


def engine_search(orig, filter_name=None, kernel_idx=0, ctus=None, want_sad_satd=False, nthreads=0):
    """What the engine returns when it filters the references itself (filter_name) or uses
    the originals (None): the oracle's search with the engine's UNAVAILABLE entries
    (engine_unavailable_mask) filled in."""
    from mipgpu import layout
    refs = None if filter_name is None else filter_frame(orig, filter_name, kernel_idx)
    res = search(orig, refs, ctus=ctus, want_sad_satd=want_sad_satd, nthreads=nthreads)
    if filter_name is not None:
        m = engine_unavailable_mask(orig, filter_name, kernel_idx)
        if ctus is not None:
            keep = np.zeros_like(m)
            keep[ctus[0] * layout.COSTS_PER_CTU:ctus[1] * layout.COSTS_PER_CTU] = True
            m &= keep
        for t in (res if want_sad_satd else (res,)):
            t[m] = layout.UNAVAILABLE
    return res
