"""Static tables: the generated header / Python table vs the reference's constants."""
import os
import subprocess
import sys

import numpy as np
import pytest

from mipgpu import layout

REF = "/root/reference"
HAVE_REF = os.path.exists(os.path.join(REF, "constants.cl"))
TOOLS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")


def test_cost_layout_totals():
    assert sum(s.ncu * s.total_modes for s in layout.SHAPES) == layout.COSTS_PER_CTU == 97840
    assert sum(s.ncu for s in layout.SHAPES) == layout.CUS_PER_CTU == 5380
    offs = [s.cost_offset for s in layout.SHAPES]
    assert offs == sorted(offs) and offs[0] == 0


def test_cu_positions_inside_ctu_and_disjoint():
    for s in layout.SHAPES:
        x, y = s.positions()
        assert (x % 4 == 0).all() and (y % 4 == 0).all()
        assert (x + s.w <= 128).all() and (y + s.h <= 128).all()
        occ = np.zeros((128, 128), np.int32)
        for xi, yi in zip(x, y):
            occ[yi:yi + s.h, xi:xi + s.w] += 1
        assert occ.max() == 1, s.name  # CUs of one shape never overlap


def test_best_modes_numpy():
    rng = np.random.default_rng(1)
    c = rng.integers(0, 1000, size=2 * 97840).astype(np.int32)
    c[5] = layout.UNAVAILABLE
    m, v = layout.best_modes(c, 2)
    assert m.shape == (2 * 5380,)
    s0 = layout.SHAPES[0]
    row = c[:s0.total_modes]
    assert m[0] == np.argmin(row) and v[0] == row.min()


@pytest.mark.skipif(not HAVE_REF, reason="reference tree not mounted")
def test_topk_numpy_statement():
    """layout.topk_modes: stable ordering, padding past a CU's modes, unavailable CUs."""
    rng = np.random.default_rng(5)
    c = rng.integers(0, 50, size=2 * layout.COSTS_PER_CTU).astype(np.int32)  # many ties
    c[layout.COSTS_PER_CTU:layout.COSTS_PER_CTU + 12] = layout.UNAVAILABLE   # CU 0 of CTU 1
    m1, v1 = layout.topk_modes(c, 2, 1)
    bm, bv = layout.best_modes(c, 2)
    assert np.array_equal(m1[:, 0], bm) and np.array_equal(v1[:, 0], bv)
    m, v = layout.topk_modes(c, 2, 32)
    s0 = layout.SHAPES[0]
    row = c[:2 * s0.modes]
    want = sorted(range(len(row)), key=lambda i: (row[i], i))
    assert list(m[0, :len(row)]) == want and list(v[0, :len(row)]) == [row[i] for i in want]
    assert (m[0, len(row):] == 0xFF).all() and (v[0, len(row):] == layout.UNAVAILABLE).all()
    assert (m[layout.CUS_PER_CTU] == 0xFF).all() and (v[layout.CUS_PER_CTU] == layout.UNAVAILABLE).all()
    assert (np.diff(v[:, :12].astype(np.int64), axis=1) >= 0).all()


def test_generated_header_matches_reference():
    """Re-derive the tables from the reference files and compare with the committed ones."""
    sys.path.insert(0, TOOLS)
    from gen_tables import render
    text, offs, c = render()
    hdr = os.path.join(os.path.dirname(TOOLS), "vvc-mip-gpu_amd", "csrc", "mip_tables.h")
    assert open(hdr).read() == text
    assert offs + [97840] == c["ALL_stridedDistortionsPerCtu"]
    # Positions re-expanded from the lattice description == ALL_X_POS / ALL_Y_POS rows.
    from refparse import parse_rows
    X = parse_rows(REF + "/constants.cl", "ALL_X_POS")
    Y = parse_rows(REF + "/constants.cl", "ALL_Y_POS")
    for s in layout.SHAPES[:46]:
        x, y = s.positions()
        assert list(x) == X[s.index][:s.ncu] and list(y) == Y[s.index][:s.ncu], s.name
    assert [s.w for s in layout.SHAPES] == c["ALL_widths"]
    assert [s.h for s in layout.SHAPES] == c["ALL_heights"]
    assert [s.ncu for s in layout.SHAPES] == c["ALL_cusPerCtu"]
    assert [s.modes for s in layout.SHAPES] == c["ALL_numPredModes"]


def _taps(name):
    hdr = open(os.path.join(os.path.dirname(TOOLS), "vvc-mip-gpu_amd", "csrc", "mip_tables.h")).read()
    line = next(l for l in hdr.splitlines() if l.startswith("#define " + name))
    return [int(v) for v in line[line.index("{") + 1:line.index("}")].split(",")]


@pytest.mark.parametrize("name,ks,n", [("MIP_TAPS_3x3", 3, 5), ("MIP_TAPS_5x5", 5, 3)])
def test_filter_kernels_are_outer_product_plus_centre(name, ks, n):
    """mip_filter.hip computes every 2-D filter as t (x) t + d * delta with t = row 0 of
    the kernel (convKernelLib, constants.cl) -- true for every kernel of the library."""
    taps = np.array(_taps(name)).reshape(n, ks, ks)
    for k in taps:
        t = k[0]
        d = k[ks // 2, ks // 2] - t[ks // 2] ** 2
        want = np.outer(t, t)
        want[ks // 2, ks // 2] += d
        assert np.array_equal(k, want) and (k == k.T).all()


def test_torch_synth_matches_numpy_generator():
    """bench.py generates its frames with torch on the GPU (synth_frames_torch); they must be
    the frames of the numpy / C generator (large seeds: the uint64 wrap-around)."""
    import torch  # noqa: F401
    from mipgpu.synth import synth_frames, synth_frames_torch
    for kind, seed in ((0, 0x1080), (0, 0x1080 + 7 * 1000003), (1, 0xFFFFFFFFFFF0), (2, 5)):
        a = synth_frames(136, 72, 2, seed, kind)
        b = synth_frames_torch(136, 72, 2, seed, kind).numpy().astype(np.uint16)
        assert np.array_equal(a, b), (kind, seed)

