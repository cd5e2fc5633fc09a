"""Cost-table layout of the MIP search, mirroring the reference host tables.

The cost table of a frame is int32[nCTUs * 97840], indexed
``ctu*97840 + shape.cost_offset + cu*2*modes + mode`` exactly like the reference's
``ALL_stridedDistortionsPerCtu`` layout (constants.h:1558-1631) that
``exportAllDistortionValues_File`` walks (main_aux_functions.h:735-798).
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache

import numpy as np

from ._tables import SHAPES as _RAW

COSTS_PER_CTU = 97840
CUS_PER_CTU = 5380
UNAVAILABLE = 0x7FFFFFFF
NUM_SHAPES = 47


@dataclass(frozen=True)
class Shape:
    index: int
    name: str
    w: int
    h: int
    size_id: int
    modes: int          # MIP modes without transposition (6 / 8 / 16)
    ncols: int
    nrows: int
    ncu: int
    xb: int
    xs: int
    xd: int
    yb: int
    ys: int
    yd: int
    cost_offset: int

    @property
    def total_modes(self) -> int:
        return 2 * self.modes

    @staticmethod
    def _axis(base, step, dual, n):
        i = np.arange(n)
        if dual:
            return base + (i // 2) * step + (i % 2) * dual
        return base + i * step

    def positions(self):
        """(x, y) of every CU of the shape inside the CTU, CU order."""
        xs = self._axis(self.xb, self.xs, self.xd, self.ncols)
        ys = self._axis(self.yb, self.ys, self.yd, self.nrows)
        cu = np.arange(self.ncu)
        return xs[cu % self.ncols], ys[cu // self.ncols]


SHAPES = tuple(Shape(i, *row) for i, row in enumerate(_RAW))
SHAPE_BY_NAME = {s.name: s for s in SHAPES}


def ctu_grid(width: int, height: int):
    """(ctu columns, ctu rows), intra.cl:31-33."""
    return (width + 127) // 128, (height + 127) // 128


def num_ctus(width: int, height: int) -> int:
    c, r = ctu_grid(width, height)
    return c * r


@lru_cache(maxsize=None)
def ctu_entries():
    """Per-entry metadata of ONE CTU's 97840 costs: shape, cu, mode, x, y, w, h."""
    shape = np.empty(COSTS_PER_CTU, np.int16)
    cu = np.empty(COSTS_PER_CTU, np.int16)
    mode = np.empty(COSTS_PER_CTU, np.int16)
    x = np.empty(COSTS_PER_CTU, np.int16)
    y = np.empty(COSTS_PER_CTU, np.int16)
    w = np.empty(COSTS_PER_CTU, np.int16)
    h = np.empty(COSTS_PER_CTU, np.int16)
    for s in SHAPES:
        m = s.total_modes
        n = s.ncu * m
        sl = slice(s.cost_offset, s.cost_offset + n)
        px, py = s.positions()
        shape[sl] = s.index
        cu[sl] = np.repeat(np.arange(s.ncu), m)
        mode[sl] = np.tile(np.arange(m), s.ncu)
        x[sl] = np.repeat(px, m)
        y[sl] = np.repeat(py, m)
        w[sl] = s.w
        h[sl] = s.h
    for a in (shape, cu, mode, x, y, w, h):
        a.setflags(write=False)
    return dict(shape=shape, cu=cu, mode=mode, x=x, y=y, w=w, h=h)


def cu_defined(width: int, height: int, x, y, w, h):
    """Does the reference define the cost of the CU at frame position (x, y)?

    The reference reads samples by linear index y' * W + x' (intra.cl:100, 106, 236, 242,
    718): a CU right of the frame reads the next row's samples, deterministically, as long
    as every index stays below W * H; its largest index is its bottom-right original sample.
    CUs with y + h > H are skipped by initBoundaries (stale LDS, intra.cl:96-98, 232-234).
    """
    y = np.asarray(y, np.int64)
    return (y + h <= height) & ((y + h - 1) * width + x + w - 1 < width * height)


def available_mask(width: int, height: int) -> np.ndarray:
    """Boolean mask over a frame's cost table: True where the reference defines the cost
    (cu_defined); this engine writes UNAVAILABLE everywhere else."""
    e = ctu_entries()
    cols, rows = ctu_grid(width, height)
    ctu = np.arange(cols * rows)
    cx = (128 * (ctu % cols))[:, None]
    cy = (128 * (ctu // cols))[:, None]
    ok = cu_defined(width, height, cx + e["x"][None, :].astype(np.int64), cy + e["y"][None, :].astype(np.int64),
                    e["w"][None, :], e["h"][None, :])
    return ok.reshape(-1)


@lru_cache(maxsize=None)
def _entry_cu():
    """CU index (CU order inside the CTU) of each of the 97840 cost entries."""
    prefix = np.cumsum([0] + [s.ncu for s in SHAPES])
    e = ctu_entries()
    return (prefix[e["shape"]] + e["cu"]).astype(np.int32)


def expand_cu_mask(cu_mask: np.ndarray, nctus: int) -> np.ndarray:
    """Per-CU bool mask (nctus * 5380, CU order) -> per-cost-entry mask (nctus * 97840)."""
    m = np.asarray(cu_mask, bool).reshape(nctus, CUS_PER_CTU)
    return m[:, _entry_cu()].reshape(-1)


def cu_count(nctus: int) -> int:
    return nctus * CUS_PER_CTU


def best_modes(costs: np.ndarray, nctus: int):
    """Per-CU argmin over modes (ties -> lowest mode), 0xff for unavailable CUs."""
    costs = costs.reshape(nctus, COSTS_PER_CTU)
    modes_out, cost_out = [], []
    for s in SHAPES:
        blk = costs[:, s.cost_offset:s.cost_offset + s.ncu * s.total_modes].reshape(nctus, s.ncu, s.total_modes)
        am = blk.argmin(axis=2)
        mn = np.take_along_axis(blk, am[..., None], axis=2)[..., 0]
        am = np.where(mn == UNAVAILABLE, 0xFF, am)
        modes_out.append(am.astype(np.uint8))
        cost_out.append(mn.astype(np.int32))
    return np.concatenate(modes_out, axis=1).reshape(-1), np.concatenate(cost_out, axis=1).reshape(-1)


def topk_modes(costs: np.ndarray, nctus: int, k: int):
    """Per-CU decision lists (numpy statement of mip_topk_device): the k lowest-cost modes
    in increasing cost order, ties to the lower mode; 0xff / UNAVAILABLE past the CU's
    modes and for unavailable CUs.  Returns (modes uint8, costs int32), [nctus*5380, k]."""
    costs = costs.reshape(nctus, COSTS_PER_CTU)
    modes_out, cost_out = [], []
    for s in SHAPES:
        blk = costs[:, s.cost_offset:s.cost_offset + s.ncu * s.total_modes].reshape(nctus, s.ncu, s.total_modes)
        order = np.argsort(blk, axis=2, kind="stable")[..., :k]
        val = np.take_along_axis(blk, order, axis=2)
        pad = k - order.shape[2]
        if pad > 0:
            order = np.concatenate([order, np.full(order.shape[:2] + (pad,), 0xFF)], axis=2)
            val = np.concatenate([val, np.full(val.shape[:2] + (pad,), UNAVAILABLE)], axis=2)
        dead = blk[..., :1] == UNAVAILABLE
        order = np.where(dead, 0xFF, order)
        val = np.where(dead, UNAVAILABLE, val)
        modes_out.append(order.astype(np.uint8))
        cost_out.append(val.astype(np.int32))
    return (np.concatenate(modes_out, axis=1).reshape(-1, k), np.concatenate(cost_out, axis=1).reshape(-1, k))


BINARY_LOG_MAGIC = 0x4350494D  # "MIPC"


def read_binary_log(path: str):
    """Read a CLI --BinaryLog file: dict with width, height, frames and 'cost' (and 'sad',
    'satd' when logged) as int32 [frames, nCTUs*97840] arrays (memory-mapped)."""
    hdr = np.fromfile(path, dtype="<u4", count=8)
    if hdr.size != 8 or hdr[0] != BINARY_LOG_MAGIC or hdr[1] != 1:
        raise ValueError(f"{path}: not a version-1 MIP cost log")
    w, h, n, per, flags = (int(v) for v in hdr[2:7])
    if per != num_ctus(w, h) * COSTS_PER_CTU:
        raise ValueError(f"{path}: {per} entries per frame do not match {w}x{h}")
    names = ["cost"] + (["sad", "satd"] if flags & 1 else [])
    mm = np.memmap(path, dtype="<i4", mode="r", offset=32, shape=(len(names), n, per))
    out = {"width": w, "height": h, "frames": n}
    for i, k in enumerate(names):
        out[k] = mm[i]
    return out
