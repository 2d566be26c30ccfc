"""ctypes wrapper over the CPU oracle (``oracle/liboracle.so``).

TEST INFRASTRUCTURE ONLY.  This module restates Redis / RedisBloom arithmetic
(see ``sketch_oracle.h`` for the upstream routines and the reference call
sites it follows) and is the checker for the HIP product path.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it; the product package never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

HLL_REGISTERS = 16384
HLL_DENSE_BYTES = 12288
OPT_NOROUND = 1
OPT_FORCE64 = 4
OPT_NO_SCALING = 8

_lib = None


def build() -> str:
    """Compile liboracle.so with gcc (no GPU involved)."""
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
        os.path.join(_HERE, "sketch_oracle.c")
    ):
        build()
    L = C.CDLL(_LIB_PATH)
    u8p, u32p, u64p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)
    L.orc_murmur64a.restype = C.c_uint64
    L.orc_murmur64a.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
    L.orc_smhasher_verification.restype = C.c_uint32
    L.orc_hll_patlen.restype = C.c_int
    L.orc_hll_patlen.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_long)]
    L.orc_hll_add.restype = C.c_int
    L.orc_hll_add.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    L.orc_hll_count.restype = C.c_uint64
    L.orc_hll_count.argtypes = [C.c_void_p]
    L.orc_hll_estimate.restype = C.c_uint64
    L.orc_hll_estimate.argtypes = [C.c_void_p]
    L.orc_hll_merge.argtypes = [C.c_void_p, C.c_void_p]
    L.orc_hll_dense_encode.argtypes = [C.c_void_p, C.c_void_p]
    L.orc_hll_dense_decode.argtypes = [C.c_void_p, C.c_void_p]
    L.orc_hll_decode_string.restype = C.c_int
    L.orc_hll_decode_string.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p]
    L.orc_hll_tau.restype = C.c_double
    L.orc_hll_tau.argtypes = [C.c_double]
    L.orc_hll_sigma.restype = C.c_double
    L.orc_hll_sigma.argtypes = [C.c_double]
    L.orc_chain_new.restype = C.c_void_p
    L.orc_chain_new.argtypes = [C.c_uint64, C.c_double, C.c_uint, C.c_uint]
    L.orc_chain_free.argtypes = [C.c_void_p]
    L.orc_chain_add.restype = C.c_int
    L.orc_chain_add.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    L.orc_chain_check.restype = C.c_int
    L.orc_chain_check.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, u64p]
    L.orc_chain_nlinks.restype = C.c_int
    L.orc_chain_nlinks.argtypes = [C.c_void_p]
    L.orc_chain_size.restype = C.c_uint64
    L.orc_chain_size.argtypes = [C.c_void_p]
    L.orc_chain_link_info.restype = C.c_int
    L.orc_chain_link_info.argtypes = [C.c_void_p, C.c_int, u64p, u64p, u64p,
                                      C.POINTER(C.c_int), u64p, C.POINTER(C.c_double)]
    L.orc_chain_link_bits.restype = C.c_void_p
    L.orc_chain_link_bits.argtypes = [C.c_void_p, C.c_int]
    L.orc_chain_madd.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    L.orc_chain_mexists.restype = C.c_uint64
    L.orc_chain_mexists.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    L.orc_process_swipes.restype = C.c_uint64
    L.orc_process_swipes.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_uint64, C.c_void_p, u64p]
    L.orc_process_swipes_mt.restype = C.c_uint64
    L.orc_process_swipes_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_uint64, C.c_void_p, u64p, C.c_int]
    L.orc_hll_madd.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                               C.c_void_p]
    L.orc_chain_dump_header.restype = C.c_size_t
    L.orc_chain_dump_header.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.orc_chain_dump_chunk.restype = C.c_size_t
    L.orc_chain_dump_chunk.argtypes = [C.c_void_p, C.POINTER(C.c_longlong), C.c_size_t,
                                       C.POINTER(C.c_void_p)]
    L.orc_chain_from_header.restype = C.c_void_p
    L.orc_chain_from_header.argtypes = [C.c_char_p, C.c_size_t]
    L.orc_chain_load_chunk.restype = C.c_int
    L.orc_chain_load_chunk.argtypes = [C.c_void_p, C.c_longlong, C.c_char_p, C.c_size_t]
    _lib = L
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def pack(items) -> tuple[np.ndarray, np.ndarray]:
    """bytes items -> (u8 bytes, u32 offsets[n+1])."""
    lens = np.fromiter((len(x) for x in items), dtype=np.uint64, count=len(items))
    offs = np.zeros(len(items) + 1, dtype=np.uint32)
    np.cumsum(lens, out=offs[1:], dtype=np.uint64) if len(items) else None
    buf = np.frombuffer(b"".join(items), dtype=np.uint8).copy() if items else np.zeros(0, np.uint8)
    return buf, offs


def murmur64a(data: bytes, seed: int) -> int:
    return lib().orc_murmur64a(data, len(data), seed)


def smhasher_verification() -> int:
    return lib().orc_smhasher_verification()


class HLL:
    """Raw-register HLL (Redis HLL_RAW view of a dense/sparse key)."""

    def __init__(self, regs: np.ndarray | None = None):
        self.regs = np.zeros(HLL_REGISTERS, np.uint8) if regs is None else regs.astype(np.uint8).copy()

    def add(self, *elems: bytes) -> int:
        L = lib()
        ch = 0
        for e in elems:
            ch |= L.orc_hll_add(_ptr(self.regs), e, len(e))
        return ch

    def count(self) -> int:
        return lib().orc_hll_count(_ptr(self.regs))

    def merge(self, other: "HLL") -> None:
        lib().orc_hll_merge(_ptr(self.regs), _ptr(other.regs))

    def dense(self) -> bytes:
        out = np.zeros(HLL_DENSE_BYTES, np.uint8)
        lib().orc_hll_dense_encode(_ptr(self.regs), _ptr(out))
        return out.tobytes()


def hll_estimate(histo: np.ndarray) -> int:
    h = np.ascontiguousarray(histo, dtype=np.int32)
    assert h.shape == (64,)
    return lib().orc_hll_estimate(_ptr(h))


def hll_count_regs(regs: np.ndarray) -> int:
    r = np.ascontiguousarray(regs, dtype=np.uint8)
    return lib().orc_hll_count(_ptr(r))


def hll_decode_string(s: bytes) -> np.ndarray | None:
    regs = np.zeros(HLL_REGISTERS, np.uint8)
    rc = lib().orc_hll_decode_string(s, len(s), _ptr(regs))
    return regs if rc == 0 else None


MAX_SCANDUMP_SIZE = 10 * 1024 * 1024  # rebloom.c MAX_SCANDUMP_SIZE [recall]


class Chain:
    """RedisBloom scalable chain (SB_NewChain options as rebloom.c uses)."""

    def __init__(self, capacity: int, error: float, expansion: int = 2, nonscaling: bool = False,
                 _ptr_=None):
        if _ptr_ is not None:
            self.p = _ptr_
            return
        opts = OPT_FORCE64 | OPT_NOROUND | (OPT_NO_SCALING if nonscaling else 0)
        self.p = lib().orc_chain_new(capacity, error, opts, expansion)
        if not self.p:
            raise ValueError("orc_chain_new failed")

    # ---- BF.SCANDUMP / BF.LOADCHUNK (RedisBloom src/sb.c, restated in C)
    def scandump(self, it: int, max_chunk: int = MAX_SCANDUMP_SIZE) -> tuple[int, bytes]:
        """BF.SCANDUMP key it -> (next iterator, data)."""
        L = lib()
        if it == 0:
            n = L.orc_chain_dump_header(self.p, None, 0)
            out = np.zeros(n, np.uint8)
            L.orc_chain_dump_header(self.p, _ptr(out), n)
            return 1, out.tobytes()
        cur, data = C.c_longlong(it), C.c_void_p()
        n = L.orc_chain_dump_chunk(self.p, C.byref(cur), max_chunk, C.byref(data))
        return cur.value, (C.string_at(data.value, n) if n else b"")

    def scandump_all(self, max_chunk: int = MAX_SCANDUMP_SIZE) -> list[tuple[int, bytes]]:
        """Every (iterator, chunk) pair a client's SCANDUMP loop collects, header first."""
        out, it = [], 0
        while True:
            it, data = self.scandump(it, max_chunk)
            if it == 0:
                return out
            out.append((it, data))

    @classmethod
    def loadchunks(cls, chunks) -> "Chain":
        """BF.LOADCHUNK of every (iterator, chunk) pair into a new chain."""
        L = lib()
        (it0, hdr), rest = chunks[0], chunks[1:]
        assert it0 == 1
        p = L.orc_chain_from_header(hdr, len(hdr))
        if not p:
            raise ValueError("ERR received bad data")
        ch = cls(0, 0, _ptr_=p)
        for it, data in rest:
            rc = L.orc_chain_load_chunk(p, it, data, len(data))
            if rc:
                raise ValueError(f"LOADCHUNK rc {rc}")
        return ch

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_chain_free(self.p)
            self.p = None

    def add(self, item: bytes) -> int:
        return lib().orc_chain_add(self.p, item, len(item))

    def exists(self, item: bytes) -> int:
        return lib().orc_chain_check(self.p, item, len(item), None)

    def madd_packed(self, buf: np.ndarray, offs: np.ndarray) -> np.ndarray:
        n = len(offs) - 1
        out = np.zeros(n, np.int8)
        lib().orc_chain_madd(self.p, _ptr(buf), _ptr(offs), n, _ptr(out))
        return out

    def mexists_packed(self, buf: np.ndarray, offs: np.ndarray) -> tuple[np.ndarray, int]:
        n = len(offs) - 1
        out = np.zeros(n, np.uint8)
        probes = lib().orc_chain_mexists(self.p, _ptr(buf), _ptr(offs), n, _ptr(out))
        return out, probes

    @property
    def nlinks(self) -> int:
        return lib().orc_chain_nlinks(self.p)

    @property
    def size(self) -> int:
        return lib().orc_chain_size(self.p)

    def link_info(self, i: int) -> dict:
        e, by, bi, sz = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        h, err = C.c_int(), C.c_double()
        rc = lib().orc_chain_link_info(self.p, i, C.byref(e), C.byref(by), C.byref(bi),
                                       C.byref(h), C.byref(sz), C.byref(err))
        if rc:
            raise IndexError(i)
        return dict(entries=e.value, bytes=by.value, bits=bi.value, hashes=h.value,
                    size=sz.value, error=err.value)

    def link_bits(self, i: int) -> np.ndarray:
        info = self.link_info(i)
        p = lib().orc_chain_link_bits(self.p, i)
        return np.ctypeslib.as_array((C.c_uint8 * info["bytes"]).from_address(p)).copy()


def process_swipes(chain: Chain | None, regs: np.ndarray, slot: np.ndarray, buf: np.ndarray,
                   offs: np.ndarray, threads: int = 1) -> tuple[np.ndarray, int, int]:
    """Per-event loop of attendance_processor.py:100-137 (no transport).

    regs: (nkeys, 16384) u8, updated in place.  Returns (valid u8[n], nvalid, probes).
    threads > 1 runs orc_process_swipes_mt (same results, host-thread timing)."""
    n = len(offs) - 1
    out = np.zeros(n, np.uint8)
    probes = C.c_uint64(0)
    assert regs.dtype == np.uint8 and regs.flags.c_contiguous
    slot = np.ascontiguousarray(slot, np.uint32)
    if threads > 1:
        nvalid = lib().orc_process_swipes_mt(chain.p if chain else None, _ptr(regs), _ptr(slot),
                                             _ptr(buf), _ptr(offs), n, _ptr(out),
                                             C.byref(probes), int(threads))
    else:
        nvalid = lib().orc_process_swipes(chain.p if chain else None, _ptr(regs), _ptr(slot),
                                          _ptr(buf), _ptr(offs), n, _ptr(out), C.byref(probes))
    return out, nvalid, probes.value


def hll_madd(regs: np.ndarray, slot: np.ndarray, buf: np.ndarray, offs: np.ndarray) -> np.ndarray:
    n = len(offs) - 1
    out = np.zeros(n, np.uint8)
    lib().orc_hll_madd(_ptr(regs), _ptr(np.ascontiguousarray(slot, np.uint32)), _ptr(buf),
                       _ptr(offs), n, _ptr(out))
    return out
