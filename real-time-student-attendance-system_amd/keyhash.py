"""MurmurHash64A in Python for host-side key routing (shard = hash(key) mod
world).  Same function the device uses for ids (sketch_common.h), applied to
Redis key names; not on the per-swipe path."""
from __future__ import annotations

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
