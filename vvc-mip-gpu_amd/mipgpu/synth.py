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
