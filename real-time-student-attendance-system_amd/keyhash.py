"""MurmurHash64A in Python for host-side key routing (shard = hash(key) mod
world).  Same function the device uses for ids (sketch_common.h), applied to
Redis key names; not on the per-swipe path.

``murmur64a_many`` hashes a whole key universe at once (numpy, keys grouped
by length): a C5 rollup names 1.825 M lecture-day keys, which the scalar
loop would take seconds over."""
from __future__ import annotations

from typing import Sequence

import numpy as np

_M = 0xC6A4A7935BD1E995
_MASK = (1 << 64) - 1


def murmur64a(data: bytes, seed: int) -> int:
    n = len(data)
    h = (seed ^ (n * _M)) & _MASK
    nb = n // 8
    for i in range(nb):
        k = int.from_bytes(data[8 * i:8 * i + 8], "little")
        k = (k * _M) & _MASK
        k ^= k >> 47
        k = (k * _M) & _MASK
        h ^= k
        h = (h * _M) & _MASK
    rem = n & 7
    if rem:
        h ^= int.from_bytes(data[8 * nb:], "little")
        h = (h * _M) & _MASK
    h ^= h >> 47
    h = (h * _M) & _MASK
    h ^= h >> 47
    return h


def _murmur_same_len(rows: np.ndarray, seed: int) -> np.ndarray:
    """MurmurHash64A of every row of a [m, n] uint8 array (all of length n)."""
    m, n = rows.shape
    M = np.uint64(_M)
    r47 = np.uint64(47)
    h = np.full(m, (seed ^ (n * _M)) & _MASK, np.uint64)
    nb = n // 8
    with np.errstate(over="ignore"):
        if nb:
            blocks = np.ascontiguousarray(rows[:, :8 * nb]).view("<u8").reshape(m, nb)
            for i in range(nb):
                k = blocks[:, i] * M
                k ^= k >> r47
                k *= M
                h ^= k
                h *= M
        rem = n & 7
        if rem:
            tail = np.zeros((m, 8), np.uint8)
            tail[:, :rem] = rows[:, 8 * nb:]
            h ^= tail.view("<u8").reshape(m)
            h *= M
        h ^= h >> r47
        h *= M
        h ^= h >> r47
    return h


def murmur64a_many(keys: Sequence[bytes], seed: int) -> np.ndarray:
    """MurmurHash64A(key, seed) of every key (uint64 array, input order)."""
    out = np.empty(len(keys), np.uint64)
    if not len(keys):
        return out
    lens = np.fromiter((len(k) for k in keys), np.int64, len(keys))
    for n in np.unique(lens):
        idx = np.nonzero(lens == n)[0]
        rows = np.frombuffer(b"".join(keys[i] for i in idx), np.uint8).reshape(len(idx), int(n))
        out[idx] = _murmur_same_len(rows, seed)
    return out
