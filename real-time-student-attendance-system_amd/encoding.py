"""redis-py argument encoding and item packing.

redis-py's ``Encoder.encode`` turns ``bytes``/``memoryview`` into themselves,
``int``/``float`` into ``repr(value).encode()`` and ``str`` into UTF-8, and
refuses ``bool`` and anything else with ``DataError``.  The reference passes
``student_id`` as a Python ``int`` (data_generator.py:113, :143;
attendance_processor.py:104-112), so the bytes hashed by RedisBloom and Redis
are the decimal ASCII digits of the id.  ``pack`` produces the ``bytes +
offs[n+1]`` layout of the C-ABI.
"""
from __future__ import annotations

import numpy as np

from .exceptions import DataError


def encode(value) -> bytes:
    if isinstance(value, bytes):
        return value
    if isinstance(value, (bytearray, memoryview)):
        return bytes(value)
    if isinstance(value, bool):
        raise DataError("Invalid input of type: 'bool'. Convert to a bytes, string, int or "
                        "float first.")
    if isinstance(value, (int, float)):
        return repr(value).encode()
    if isinstance(value, (np.integer,)):
        return repr(int(value)).encode()
    if isinstance(value, (np.floating,)):
        return repr(float(value)).encode()
    if isinstance(value, str):
        return value.encode("utf-8")
    raise DataError(f"Invalid input of type: '{type(value).__name__}'. Convert to a bytes, "
                    "string, int or float first.")


def pack(items) -> tuple[np.ndarray, np.ndarray]:
    """Encode and pack items -> (u8 bytes, u32 offs[n+1])."""
    enc = [encode(x) for x in items]
    n = len(enc)
    offs = np.zeros(n + 1, dtype=np.uint32)
    if n:
        lens = np.fromiter((len(e) for e in enc), dtype=np.int64, count=n)
        total = int(lens.sum())
        if total >= 2**32:
            raise DataError("batch too large (>= 4 GiB of item bytes)")
        offs[1:] = np.cumsum(lens)
    buf = np.frombuffer(b"".join(enc), dtype=np.uint8) if n else np.zeros(0, np.uint8)
    return np.ascontiguousarray(buf), offs


_POW10 = np.array([10 ** k for k in range(20)], dtype=np.uint64)


def pack_ints(values) -> tuple[np.ndarray, np.ndarray]:
    """Vectorised ``pack`` for non-negative integers (decimal ASCII, as
    redis-py encodes ``int``): no Python loop over the items."""
    v = np.ascontiguousarray(values, dtype=np.uint64)
    n = v.shape[0]
    if n == 0:
        return np.zeros(0, np.uint8), np.zeros(1, np.uint32)
    nd = np.ones(n, dtype=np.int64)
    for k in range(1, 20):
        nd += (v >= _POW10[k]).astype(np.int64)
    offs = np.zeros(n + 1, dtype=np.uint32)
    offs[1:] = np.cumsum(nd)
    total = int(offs[-1])
    out = np.empty(total, dtype=np.uint8)
    maxd = int(nd.max())
    x = v.copy()
    # digit j counted from the right lands at offs[i+1]-1-j
    for j in range(maxd):
        digit = (x % np.uint64(10)).astype(np.uint8) + np.uint8(48)
        has = nd > j
        pos = offs[1:].astype(np.int64) - 1 - j
        out[pos[has]] = digit[has]
        x //= np.uint64(10)
    return out, offs
