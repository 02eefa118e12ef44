"""Deterministic synthetic-input generator (splitmix64, seed
0x7115EC0DE per config).  Pure Python for small fixtures; numpy-vectorised for
bulk batches.  Shared by tests/, bench.py and the fixture generator."""
from __future__ import annotations

import numpy as np

MASK = (1 << 64) - 1


def splitmix64(state: int):
    state = (state + 0x9E3779B97F4A7C15) & MASK
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return state, z ^ (z >> 31)


def prng_bytes(seed: int, n: int) -> bytes:
    out = bytearray()
    s = seed & MASK
    while len(out) < n:
        s, z = splitmix64(s)
        out += z.to_bytes(8, "little")
    return bytes(out[:n])


def prng_array(seed: int, nbytes: int) -> np.ndarray:
    """Vectorised splitmix64 stream: word i = mix(seed + (i+1)*golden)."""
    nw = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        idx = np.arange(1, nw + 1, dtype=np.uint64)
        z = np.uint64(seed & MASK) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes]
