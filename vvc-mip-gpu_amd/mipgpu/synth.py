"""Deterministic synthetic 10-bit frames (integer-only, identical to the C generator
in oracle/mip_oracle.c so fixtures can be regenerated anywhere from (kind, seed))."""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth_frame(width: int, height: int, seed: int, kind: int = 0) -> np.ndarray:
    """kind 0: structured (ramps + texture + block DC + noise); kind 1: uniform noise;
    kind 2: near-black noise in {0, 1, 2} (filter quotients around 1/2)."""
    y, x = np.meshgrid(np.arange(height, dtype=np.uint64), np.arange(width, dtype=np.uint64), indexing="ij")
    with np.errstate(over="ignore"):
        s = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
        h = _splitmix64(s * np.uint64(0x100000001B3) + y * np.uint64(width) + x)
    if kind == 1:
        return (h & np.uint64(1023)).astype(np.uint16)
    if kind == 2:
        return (h % np.uint64(3)).astype(np.uint16)
    hb = _splitmix64(s ^ ((y >> np.uint64(5)) << np.uint64(32)) ^ (x >> np.uint64(5)))
    xi, yi = x.astype(np.int64), y.astype(np.int64)
    ramp = (xi * 3 + yi * 5) % 512
    tp = (xi + 2 * yi) % 96
    tri = np.where(tp < 48, tp, 96 - tp) * 4
    dc = (hb & np.uint64(255)).astype(np.int64) - 128
    noise = ((h >> np.uint64(20)) & np.uint64(31)).astype(np.int64) - 16
    v = 200 + ramp + tri - 96 + dc + noise
    return np.clip(v, 0, 1023).astype(np.uint16)


def synth_frames(width: int, height: int, nframes: int, seed: int, kind: int = 0) -> np.ndarray:
    return np.stack([synth_frame(width, height, seed + f, kind) for f in range(nframes)])


def synth_frames_torch(width: int, height: int, nframes: int, seed: int, kind: int = 0, device=None):
    """synth_frames computed with torch on `device` (e.g. the GPU the bench runs on: 128
    1080p frames in well under a second instead of ~25 s of numpy), bit-identical: the
    uint64 arithmetic runs in int64 with two's-complement wrap-around and the logical right
    shifts masked (tests/test_tables.py checks it against synth_frames).  Returns int16
    [nframes, height, width] holding the 10-bit samples."""
    import torch

    def lsr(z, k):  # logical right shift of a uint64 held in int64
        return (z >> k) & ((1 << (64 - k)) - 1)

    def u64(v):  # a uint64 constant as the int64 with the same bits
        v &= 0xFFFFFFFFFFFFFFFF
        return v - (1 << 64) if v >= 1 << 63 else v

    def splitmix64(z):
        z = z + u64(0x9E3779B97F4A7C15)
        z = (z ^ lsr(z, 30)) * u64(0xBF58476D1CE4E5B9)
        z = (z ^ lsr(z, 27)) * u64(0x94D049BB133111EB)
        return z ^ lsr(z, 31)

    y = torch.arange(height, dtype=torch.int64, device=device).view(height, 1)
    x = torch.arange(width, dtype=torch.int64, device=device).view(1, width)
    pos = y * width + x
    out = torch.empty((nframes, height, width), dtype=torch.int16, device=device)
    if kind == 0:
        xi, yi = x, y
        ramp = (xi * 3 + yi * 5) % 512
        tp = (xi + 2 * yi) % 96
        tri = torch.where(tp < 48, tp, 96 - tp) * 4
        base = 200 + ramp + tri - 96
    for f in range(nframes):
        s = u64(seed + f)
        h = splitmix64(u64((seed + f) * 0x100000001B3) + pos)  # the product wraps like uint64
        if kind == 1:
            v = h & 1023
        elif kind == 2:
            v = torch.remainder(lsr(h, 1), 3) * 2 + (h & 1)  # (h mod 3) of the unsigned value
            v = torch.remainder(v, 3)
        else:
            hb = splitmix64(s ^ ((y >> 5) << 32) ^ (x >> 5))
            dc = (hb & 255) - 128
            noise = (lsr(h, 20) & 31) - 16
            v = torch.clamp(base + dc + noise, 0, 1023)
        out[f] = v.to(torch.int16)
    return out

