"""Host (numpy) Philox4x32-10 — the counter-based generator behind the fused plans' dropout masks
(csrc/kernels/bncnn.hip ``philox`` / ``keep_scale``; Keras Dropout, mnist_keras_distributed.py:106).

The device draws one Philox block per 4 consecutive elements of a [B, D] activation:
counter = (e // 4 low, e // 4 high, step, layer), key = (seed low, seed high); element e keeps its
value iff ``(word[e % 4] >> 8) / 2**24 < 1 - rate`` and is then scaled by ``1 / (1 - rate)``.
``keep_scales`` reproduces that bit for bit, so tests can pin the device mask to the published
generator (Random123 known-answer vectors) and a host oracle can apply the very same mask.
"""
from __future__ import annotations

import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """Philox4x32 with 10 rounds over arrays: ``ctr`` [..., 4] uint32, ``key`` [..., 2] uint32 ->
    [..., 4] uint32."""
    c = np.array(ctr, dtype=np.uint32, copy=True)
    k = np.array(key, dtype=np.uint32, copy=True)
    c0, c1, c2, c3 = (c[..., i].astype(np.uint64) for i in range(4))
    k0, k1 = k[..., 0].astype(np.uint64), k[..., 1].astype(np.uint64)
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0)
        k0 = (k0 + _W0) & _MASK32      # the key schedule wraps at 32 bits
        k1 = (k1 + _W1) & _MASK32
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


def keep_scales(rate: float, seed: int, step: int, layer: int, n: int) -> np.ndarray:
    """The device's dropout keep scales of elements 0..n-1 (float32: 1/(1-rate) or 0)."""
    nb = (n + 3) // 4
    blk = np.arange(nb, dtype=np.uint64)
    ctr = np.stack([(blk & _MASK32).astype(np.uint32), (blk >> np.uint64(32)).astype(np.uint32),
                    np.full(nb, step & 0xFFFFFFFF, np.uint32), np.full(nb, layer & 0xFFFFFFFF, np.uint32)], axis=-1)
    key = np.broadcast_to(np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF], np.uint32), (nb, 2))
    words = philox4x32_10(ctr, key).reshape(-1)[:n]
    keep = np.float32(1.0) - np.float32(rate)   # float32 arithmetic, as on the device
    u = (words >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return np.where(u < keep, np.float32(1.0) / keep, np.float32(0.0)).astype(np.float32)
