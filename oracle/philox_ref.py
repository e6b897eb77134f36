"""TEST INFRASTRUCTURE ONLY (the checker, never the product): numpy restatement of the Langevin
kernel's noise stream, Philox4x32-10 (Salmon et al., SC'11) + Box-Muller.

The reference draws ``torch.randn_like(x_mod)`` (KITTISampling.py:152, models/__init__.py:1411);
that stream cannot be reproduced on another device, so the product draws N(0,1) from Philox
keyed by (seed, counter) with one counter per 4 consecutive elements of the megabatch.  This
restatement pins that contract: the raw 32-bit words bit-exactly, the floats to the device
intrinsics' accuracy (__logf / __sincosf, ~1e-6 relative).
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr: np.ndarray, seed: int) -> np.ndarray:
    """ctr: uint64[n] counters -> uint32[n, 4] words (counter words (lo, hi, 0, 0), key = seed)."""
    ctr = np.asarray(ctr, dtype=np.uint64)
    z = np.zeros_like(ctr)
    return philox4x32_10_words(ctr & MASK, ctr >> np.uint64(32), z, z, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)


def philox4x32_10_words(c0, c1, c2, c3, k0, k1) -> np.ndarray:
    """The generic 4-word counter / 2-word key form (for the Random123 known-answer vectors)."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) for c in (c0, c1, c2, c3))
    k0, k1 = np.uint64(k0), np.uint64(k1)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK, lo1, (hi0 ^ c3 ^ k1) & MASK, lo0
        k0 = (k0 + np.uint64(W0)) & MASK
        k1 = (k1 + np.uint64(W1)) & MASK
    return np.stack([c0, c1, c2, c3], axis=1).astype(np.uint32)


def _u01(v):
    return (v.astype(np.float32) + np.float32(0.5)) * np.float32(2.3283064365386963e-10)


def normal(seed: int, offset: int, n: int) -> np.ndarray:
    """float32[n] (n % 4 == 0): the noise the kernel applies to elements [0, n) of a call whose
    Philox counter starts at ``offset`` (langevin.hip: normal4(seed, offset + i))."""
    assert n % 4 == 0
    r = philox4x32_10(np.arange(n // 4, dtype=np.uint64) + np.uint64(offset), seed)
    r1 = np.sqrt(np.float32(-2) * np.log(_u01(r[:, 0])))
    r2 = np.sqrt(np.float32(-2) * np.log(_u01(r[:, 2])))
    a1 = np.float32(6.283185307179586) * _u01(r[:, 1])
    a2 = np.float32(6.283185307179586) * _u01(r[:, 3])
    out = np.stack([r1 * np.cos(a1), r1 * np.sin(a1), r2 * np.cos(a2), r2 * np.sin(a2)], axis=1)
    return out.astype(np.float32).reshape(-1)
