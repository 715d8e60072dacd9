"""Synthetic, seeded inputs for the mul_mat path.

splitmix64 stream, value = (u >> 40) * 2^-24 * 2 - 1 (exact in f32), identical to
oracle/gen_fixtures.c:fill_uniform so the reference's golden vectors can be regenerated from
their seeds without storing the large f32 weight matrices.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """Outputs start..start+n-1 of the splitmix64 stream seeded with `seed`."""
    with np.errstate(over="ignore"):
        idx = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, n: int, chunk: int = 1 << 24) -> np.ndarray:
    """n float32 values in [-1, 1), bit-identical to the C generator."""
    out = np.empty(n, dtype=np.float32)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        u = splitmix64(seed, m, s)
        out[s:s + m] = (u >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0) * np.float32(2.0) - np.float32(1.0)
    return out


def cos_data(n: int = 4096, offset: float = 0.0) -> np.ndarray:
    """tests/test-quantize-fns.cpp:28-32 synthetic data 0.1 + 2*cos(i + offset) (f32 arithmetic)."""
    i = np.arange(n, dtype=np.float32) + np.float32(offset)
    return (np.float32(0.1) + np.float32(2.0) * np.cos(i).astype(np.float32)).astype(np.float32)
