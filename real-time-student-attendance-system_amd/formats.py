"""Redis on-wire formats for the sketch state.

HyperLogLog strings as Redis stores them (src/hyperloglog.c):

  header (16 B): "HYLL", encoding (0 dense, 1 sparse), 3 unused bytes,
                 8-byte little-endian cached cardinality; bit 7 of card[7] set
                 = cache invalid (HLL_INVALIDATE_CACHE)
  dense payload: 16384 x 6-bit registers packed LSB first (12288 B,
                 HLL_DENSE_SET_REGISTER)
  sparse payload: opcodes ZERO 00xxxxxx (run 1..64), XZERO 01xxxxxx yyyyyyyy
                 (run 1..16384), VAL 1vvvvvxx (value 1..32, run 1..4)

``encode_hll`` writes the canonical sparse form (maximal runs; zero runs > 64
as XZERO, as hllSparseSet splits them) when every register is <= 32 and it
fits ``sparse_max_bytes`` (server.hll_sparse_max_bytes, default 3000), else
dense -- the same promotion rule Redis applies.  Redis' own sparse bytes can
differ from the canonical form in how long VAL runs are split (they depend on
insertion history); both decode to the same registers, which is what parity is
defined on.  ``decode_hll`` accepts both encodings and rejects corrupted
strings like Redis does ("INVALIDOBJ Corrupted HLL object detected").
"""
from __future__ import annotations

import struct

import numpy as np

from .exceptions import ResponseError

HLL_REGISTERS = 16384
HLL_DENSE_BYTES = 12288
HLL_HDR = 16
HLL_DENSE, HLL_SPARSE = 0, 1
SPARSE_VAL_MAX_VALUE = 32
SPARSE_VAL_MAX_LEN = 4
SPARSE_ZERO_MAX_LEN = 64
SPARSE_XZERO_MAX_LEN = 16384
INVALIDOBJ = "INVALIDOBJ Corrupted HLL object detected"


def _header(enc: int, card: int | None) -> bytes:
    if card is None:
        c = bytearray(8)
        c[7] = 0x80  # HLL_INVALIDATE_CACHE
        cb = bytes(c)
    else:
        cb = struct.pack("<Q", int(card) & ((1 << 63) - 1))
    return b"HYLL" + bytes([enc, 0, 0, 0]) + cb


def dense_pack(regs: np.ndarray) -> bytes:
    r = np.ascontiguousarray(regs, dtype=np.uint32).reshape(-1, 4)
    bits = (r[:, 0] & 63) | ((r[:, 1] & 63) << 6) | ((r[:, 2] & 63) << 12) | ((r[:, 3] & 63) << 18)
    out = np.empty((r.shape[0], 3), np.uint8)
    out[:, 0] = bits & 0xFF
    out[:, 1] = (bits >> 8) & 0xFF
    out[:, 2] = (bits >> 16) & 0xFF
    return out.tobytes()


def dense_unpack(payload: bytes) -> np.ndarray:
    b = np.frombuffer(payload, dtype=np.uint8).reshape(-1, 3).astype(np.uint32)
    bits = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
    regs = np.empty((b.shape[0], 4), np.uint8)
    for k in range(4):
        regs[:, k] = (bits >> (6 * k)) & 63
    return regs.reshape(-1)


def sparse_pack(regs: np.ndarray) -> bytes | None:
    """Canonical sparse opcodes, or None if a register exceeds 32."""
    r = np.asarray(regs, dtype=np.uint8)
    if r.max(initial=0) > SPARSE_VAL_MAX_VALUE:
        return None
    change = np.flatnonzero(np.diff(r)) + 1
    starts = np.concatenate(([0], change))
    ends = np.concatenate((change, [HLL_REGISTERS]))
    out = bytearray()
    for s, e in zip(starts.tolist(), ends.tolist()):
        v, run = int(r[s]), e - s
        if v == 0:
            while run:
                n = min(run, SPARSE_XZERO_MAX_LEN)
                if n > SPARSE_ZERO_MAX_LEN:
                    out += bytes([0x40 | ((n - 1) >> 8), (n - 1) & 0xFF])
                else:
                    out.append(n - 1)
                run -= n
        else:
            while run:
                n = min(run, SPARSE_VAL_MAX_LEN)
                out.append(0x80 | ((v - 1) << 2) | (n - 1))
                run -= n
    return bytes(out)


def sparse_unpack(payload: bytes) -> np.ndarray:
    regs = np.zeros(HLL_REGISTERS, np.uint8)
    i = idx = 0
    n = len(payload)
    while i < n:
        op = payload[i]
        if op & 0xC0 == 0x00:
            run, val, i = (op & 0x3F) + 1, 0, i + 1
        elif op & 0xC0 == 0x40:
            if i + 1 >= n:
                raise ResponseError(INVALIDOBJ)
            run, val, i = (((op & 0x3F) << 8) | payload[i + 1]) + 1, 0, i + 2
        else:
            run, val, i = (op & 0x3) + 1, ((op >> 2) & 0x1F) + 1, i + 1
        if idx + run > HLL_REGISTERS:
            raise ResponseError(INVALIDOBJ)
        if val:
            regs[idx:idx + run] = val
        idx += run
    if idx != HLL_REGISTERS:
        raise ResponseError(INVALIDOBJ)
    return regs


def encode_hll(regs: np.ndarray, card: int | None = None, sparse_max_bytes: int = 3000) -> bytes:
    r = np.asarray(regs, dtype=np.uint8)
    if r.shape != (HLL_REGISTERS,) or r.max(initial=0) > 51:
        raise ValueError("expected 16384 registers with values <= 51")
    sp = sparse_pack(r)
    if sp is not None and len(sp) <= sparse_max_bytes:
        return _header(HLL_SPARSE, card) + sp
    return _header(HLL_DENSE, card) + dense_pack(r)


def decode_hll(s: bytes) -> np.ndarray:
    if len(s) < HLL_HDR or s[:4] != b"HYLL":
        raise ResponseError("WRONGTYPE Key is not a valid HyperLogLog string value.")
    enc = s[4]
    payload = s[HLL_HDR:]
    if enc == HLL_DENSE:
        if len(payload) != HLL_DENSE_BYTES:
            raise ResponseError(INVALIDOBJ)
        return dense_unpack(payload)
    if enc == HLL_SPARSE:
        return sparse_unpack(payload)
    raise ResponseError(INVALIDOBJ)


def cached_card(s: bytes) -> int | None:
    """The cached cardinality in the header, None if marked invalid."""
    c = s[8:16]
    if c[7] & 0x80:
        return None
    return struct.unpack("<Q", c)[0]


# ---------------------------------------------------------------------------
# RedisBloom BF.SCANDUMP / BF.LOADCHUNK header (src/sb.c dumpedChainHeader /
# dumpedChainLink, packed little-endian) -- [recall], unconfirmed on a Redis box.
# ---------------------------------------------------------------------------
_LINK = struct.Struct("<QQQddIQB")     # bytes, bits, size, error, bpe, hashes, entries, n2
_CHAIN = struct.Struct("<QIII")        # size, nfilters, options, growth
BLOOM_OPT_NOROUND, BLOOM_OPT_FORCE64, BLOOM_OPT_NO_SCALING = 1, 4, 8


def bf_dump_header(total_size: int, links: list[dict], growth: int, nonscaling: bool) -> bytes:
    opts = BLOOM_OPT_NOROUND | BLOOM_OPT_FORCE64 | (BLOOM_OPT_NO_SCALING if nonscaling else 0)
    out = _CHAIN.pack(total_size, len(links), opts, growth)
    for L in links:
        out += _LINK.pack(L["bytes"], L["bits"], L["size"], L["error"], L["bpe"], L["hashes"],
                          L["entries"], 0)
    return out


def bf_parse_header(b: bytes) -> dict:
    size, nf, opts, growth = _CHAIN.unpack_from(b, 0)
    links = []
    off = _CHAIN.size
    for _ in range(nf):
        by, bi, sz, err, bpe, h, ent, n2 = _LINK.unpack_from(b, off)
        links.append(dict(bytes=by, bits=bi, size=sz, error=err, bpe=bpe, hashes=h, entries=ent,
                          n2=n2))
        off += _LINK.size
    return {"size": size, "options": opts, "growth": growth, "links": links,
            "nonscaling": bool(opts & BLOOM_OPT_NO_SCALING)}
