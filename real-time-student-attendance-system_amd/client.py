"""SketchClient -- the redis-py call surface of the reference's hot path,
executed on MI355X through libsketch.

The reference builds one ``redis.Redis(host, port, decode_responses=True)``
client per process (attendance_processor.py:37-41, data_generator.py:45-49)
and uses exactly these calls on the validate-and-count path:

=====================================================  ====================================
reference call (file:line)                             here
=====================================================  ====================================
``execute_command('BF.EXISTS', key, id)`` (ap.py:109)  ``execute_command`` -> ske_bf_mexists
``execute_command('BF.RESERVE', key, err, cap)`` (:83) ``execute_command`` -> ske_bf_reserve
``execute_command('BF.ADD', key, id)`` (dg.py:59)      ``execute_command`` -> ske_bf_madd
``pfadd(hll_key, student_id)`` (ap.py:129)             ``pfadd`` -> ske_hll_pfadd
``pfcount(hll_key)`` (ap.py:152)                       ``pfcount`` -> ske_hll_pfcount
=====================================================  ====================================

plus the north-star surface: ``bf().reserve/add/madd/exists/mexists/info``,
``pfmerge``, ``pipeline()`` and the batched ``swipes()`` (the fused K1 kernel:
BF.EXISTS then valid-gated PFADD for a whole batch of events).

Semantics kept from Redis / RedisBloom / redis-py:
  * argument encoding as redis-py (``encoding.encode``);
  * ``BF.EXISTS``/``BF.MEXISTS`` on a missing key answer 0 (so the
    reference's probe at attendance_processor.py:78 never raises and its
    ``BF.RESERVE`` branch never runs -- reproduced, not "fixed");
  * ``BF.ADD``/``BF.MADD`` auto-create a chain (error 0.01, capacity 100,
    expansion 2); ``BF.RESERVE`` on an existing key -> ``ERR item exists``;
  * ``PFADD key`` with no elements creates the key and replies 1;
    ``PFCOUNT`` of missing keys -> 0; keys of the other type -> WRONGTYPE.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from ._lib import (BfInfo, BfLink, Context, SketchLibError, SKE_MEM_DEVICE, SKE_MEM_HOST,
                   HLL_DENSE_BYTES, HLL_REGISTERS)
from . import formats
from .encoding import encode, pack
from .exceptions import DataError, ResponseError, WRONGTYPE

BF_TYPE_NAME = "MBbloom--"  # RedisBloom's module type name (TYPE reply)
_DEFAULT_ERROR = 0.01       # rebloom.c BFDefaultErrorRate
_DEFAULT_CAPACITY = 100     # rebloom.c BFDefaultInitCapacity
_DEFAULT_EXPANSION = 2      # rebloom.c BFDefaultExpansion


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _err(e: SketchLibError) -> ResponseError:
    return ResponseError(str(e))


class KeySpace:
    """Key name -> device object (Bloom fid or HLL register-slab slot)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self.kind: dict[bytes, str] = {}
        self.fid: dict[bytes, int] = {}
        self.slot: dict[bytes, int] = {}
        self._free_fids = list(range(_lib.SKE_MAX_FILTERS - 1, -1, -1))
        self._free_slots: list[int] = []
        self._next_slot = 0
        self._slot_key: dict[int, bytes] = {}
        self.slots_released = 0  # bumps whenever an HLL slot is freed (ingest key table)
        # README day keys <stem>:YYYY-MM-DD by stem (the key minus its day),
        # kept with the table: a lecture's day keys without a scan
        self.day_keys: dict[bytes, set] = {}

    @staticmethod
    def _day_stem(key: bytes):
        """The stem of a README-form day key <stem>:YYYY-MM-DD, else None."""
        if len(key) > 11 and key[-11] == 0x3A and key[-3] == key[-6] == 0x2D and \
                key[-10:-6].isdigit() and key[-5:-3].isdigit() and key[-2:].isdigit():
            return key[:-11]
        return None

    def _index(self, key: bytes, add: bool) -> None:
        stem = self._day_stem(key)
        if stem is None:
            return
        if add:
            self.day_keys.setdefault(stem, set()).add(key)
        else:
            ks = self.day_keys.get(stem)
            if ks is not None:
                ks.discard(key)
                if not ks:
                    del self.day_keys[stem]

    def type_of(self, key: bytes) -> str | None:
        return self.kind.get(key)

    def expect(self, key: bytes, kind: str) -> bool:
        """True if the key exists with this kind, False if missing; raises
        WRONGTYPE if it holds the other kind."""
        k = self.kind.get(key)
        if k is None:
            return False
        if k != kind:
            raise ResponseError(WRONGTYPE)
        return True

    def new_fid(self, key: bytes) -> int:
        if not self._free_fids:
            raise ResponseError("ERR too many Bloom filters on this device")
        f = self._free_fids.pop()
        self.kind[key] = "bf"
        self.fid[key] = f
        return f

    def new_slot(self, key: bytes) -> int:
        if self._free_slots:
            s = self._free_slots.pop()
        else:
            s = self._next_slot
            self._next_slot += 1
            if s >= self.ctx.lib.ske_hll_capacity(self.ctx.ptr):
                self.ctx.call("ske_hll_reserve", s + 1)
        self.kind[key] = "hll"
        self.slot[key] = s
        self._slot_key[s] = key
        self._index(key, True)
        return s

    def bind(self, key: bytes, slot: int) -> None:
        """Name an HLL key at a given slab slot without touching its registers:
        a multi-GPU job's key map (distributed.KeyMap.bind) fixes the local
        slot of every key its rank owns, and K1 writes those slots directly."""
        slot = int(slot)
        if self.kind.get(key, "hll") != "hll":
            raise ResponseError(WRONGTYPE)
        have = self.slot.get(key)
        if have is not None:
            if have != slot:
                raise ResponseError(f"ERR key already bound to slot {have}")
            return
        if slot in self._slot_key:
            raise ResponseError(f"ERR slot {slot} already holds another key")
        if slot >= self.ctx.lib.ske_hll_capacity(self.ctx.ptr):
            self.ctx.call("ske_hll_reserve", slot + 1)
        if slot >= self._next_slot:
            self._free_slots.extend(range(slot - 1, self._next_slot - 1, -1))
            self._next_slot = slot + 1
        else:
            self._free_slots.remove(slot)
        self.kind[key] = "hll"
        self.slot[key] = slot
        self._slot_key[slot] = key
        self._index(key, True)

    def drop(self, key: bytes) -> bool:
        k = self.kind.pop(key, None)
        if k == "bf":
            f = self.fid.pop(key)
            self.ctx.call("ske_bf_free", f)
            self._free_fids.append(f)
        elif k == "hll":
            s = self.slot.pop(key)
            self._slot_key.pop(s, None)
            self._index(key, False)
            self.ctx.call("ske_hll_clear", s)  # a reused slot starts empty
            self._free_slots.append(s)
            self.slots_released += 1
        return k is not None

    def release_unused_slot(self, key: bytes) -> None:
        """Undo new_slot() for a key that no command ended up creating (its
        registers were never written)."""
        s = self.slot.pop(key)
        self._slot_key.pop(s, None)
        self._index(key, False)
        del self.kind[key]
        self._free_slots.append(s)
        self.slots_released += 1


def _sc(b: int) -> int:
    """a byte as C's (signed) char, as Redis compares range bounds"""
    return b - 256 if b >= 128 else b


def redis_glob(pattern: bytes, string: bytes, _nest: int = 0) -> bool:
    """Redis' SCAN / KEYS MATCH rule, restated from redis ``src/util.c``
    ``stringmatchlen`` (case-sensitive; no Redis in this image, so parity is
    unpinned -- tests/test_encoding.py holds the cases): ``*`` any run, ``?``
    one byte, ``[...]`` a class with ``^`` negation, ``a-z`` ranges (bounds
    swapped when reversed) and ``\\`` escapes, ``\\`` escaping the next
    pattern byte outside a class.  Python's fnmatch differs (``[!...]``, no
    escapes)."""
    p, s = pattern, string
    pi, si = 0, 0
    if _nest > 1000:
        return False
    while pi < len(p) and si < len(s):
        c = p[pi]
        if c == 0x2A:  # '*'
            while pi + 1 < len(p) and p[pi + 1] == 0x2A:
                pi += 1
            if pi + 1 == len(p):
                return True
            while si < len(s):
                if redis_glob(p[pi + 1:], s[si:], _nest + 1):
                    return True
                si += 1
            return False
        elif c == 0x3F:  # '?'
            si += 1
        elif c == 0x5B:  # '['
            pi += 1
            neg = pi < len(p) and p[pi] == 0x5E  # '^'
            if neg:
                pi += 1
            match = False
            while True:
                if pi < len(p) and p[pi] == 0x5C and len(p) - pi >= 2:  # '\\'
                    pi += 1
                    if p[pi] == s[si]:
                        match = True
                elif pi < len(p) and p[pi] == 0x5D:  # ']'
                    break
                elif pi >= len(p):
                    pi -= 1
                    break
                elif len(p) - pi >= 3 and p[pi + 1] == 0x2D:  # 'a-z'
                    lo, hi, ch = _sc(p[pi]), _sc(p[pi + 2]), _sc(s[si])
                    if lo > hi:
                        lo, hi = hi, lo
                    pi += 2
                    if lo <= ch <= hi:
                        match = True
                elif p[pi] == s[si]:
                    match = True
                pi += 1
            if neg:
                match = not match
            if not match:
                return False
            si += 1
        else:
            if c == 0x5C and len(p) - pi >= 2:  # an escaped byte
                pi += 1
            if p[pi] != s[si]:
                return False
            si += 1
        pi += 1
        if si == len(s):
            while pi < len(p) and p[pi] == 0x2A:
                pi += 1
            break
    return pi == len(p) and si == len(s)


class SketchClient:
    """Drop-in for ``redis.Redis`` on the reference's Bloom + HLL calls."""

    def __init__(self, host: str = "localhost", port: int = 6379, db: int = 0,
                 decode_responses: bool = False, device: int = 0,
                 context: Context | None = None, **_ignored):
        self.ctx = context if context is not None else Context(device)
        self.decode_responses = decode_responses
        self.keys = KeySpace(self.ctx)
        self.host, self.port, self.db = host, port, db

    # ------------------------------------------------------------ helpers
    _kt_state = None  # (slots released, key form, prefix) the device key table was built under

    def _ok(self):
        return "OK" if self.decode_responses else b"OK"

    def _s(self, text: str):
        return text if self.decode_responses else text.encode()

    def close(self) -> None:
        pass  # the device context lives as long as the client object

    def ping(self) -> bool:
        return True

    # ------------------------------------------------------------ generic keys
    def delete(self, *names) -> int:
        return sum(self.keys.drop(encode(n)) for n in names)

    def exists(self, *names) -> int:
        return sum(encode(n) in self.keys.kind for n in names)

    def scan_iter(self, match=None, count=None, _type=None):
        """SCAN over the key table, redis-py's iterator form (one pass, sorted;
        MATCH in Redis' own glob dialect, ``redis_glob``).  (redis-py's
        ``keys()`` is not offered: ``self.keys`` is the key table.)"""
        pat = encode(match if match is not None else "*")
        every = pat == b"*"  # SCAN's own bypass (the glob rule alone would skip an empty key name)
        for k in sorted(self.keys.kind):
            if (every or redis_glob(pat, k)) and (_type is None or self.keys.kind[k] == {"string": "hll", "MBbloom--": "bf"}.get(
                    _type, _type)):
                yield k.decode() if self.decode_responses else k

    def day_keys(self, stem) -> list:
        """The README-form day keys <stem>:YYYY-MM-DD that exist (sorted),
        from the key table's index -- no scan over every key."""
        ks = sorted(self.keys.day_keys.get(encode(stem), ()))
        return [k.decode() for k in ks] if self.decode_responses else ks

    def type(self, name):
        k = self.keys.type_of(encode(name))
        return self._s({"bf": BF_TYPE_NAME, "hll": "string", None: "none"}[k])

    def flushall(self, *_a, **_k) -> bool:
        for key in list(self.keys.kind):
            self.keys.drop(key)
        return True

    flushdb = flushall

    # ------------------------------------------------------------ Bloom
    def _bf_reserve(self, key: bytes, error_rate, capacity, expansion=None, nonscaling=False):
        try:
            err = float(error_rate)
        except (TypeError, ValueError):
            raise ResponseError("ERR bad error rate")
        try:
            cap = int(capacity)
        except (TypeError, ValueError):
            raise ResponseError("ERR bad capacity")
        if not (0 < err < 1):
            raise ResponseError("ERR (0 < error rate range < 1)")
        if cap <= 0:
            raise ResponseError("ERR (capacity should be larger than 0)")
        exp = _DEFAULT_EXPANSION if expansion is None else int(expansion)
        if exp < 1 and not nonscaling:
            raise ResponseError("ERR expansion should be greater or equal to 1")
        if key in self.keys.kind:
            if self.keys.kind[key] != "bf":
                raise ResponseError(WRONGTYPE)
            raise ResponseError("ERR item exists")
        f = self.keys.new_fid(key)
        try:
            self.ctx.call("ske_bf_reserve", f, err, cap, exp, 1 if nonscaling else 0)
        except SketchLibError as e:
            self.keys.kind.pop(key, None)
            self.keys.fid.pop(key, None)
            self.keys._free_fids.append(f)
            raise _err(e)
        return self._ok()

    def _bf_fid_for_add(self, key: bytes) -> int:
        if self.keys.expect(key, "bf"):
            return self.keys.fid[key]
        f = self.keys.new_fid(key)
        # rebloom.c: BF.ADD / BF.MADD on a missing key create a default chain
        self.ctx.call("ske_bf_reserve", f, _DEFAULT_ERROR, _DEFAULT_CAPACITY, _DEFAULT_EXPANSION, 0)
        return f

    def bf_madd_packed(self, key, buf: np.ndarray, offs: np.ndarray) -> np.ndarray:
        """BF.MADD over a packed batch; returns int8 replies (1 / 0 / -2 full)."""
        key = encode(key)
        f = self._bf_fid_for_add(key)
        n = len(offs) - 1
        out = np.zeros(n, np.int8)
        if n:
            self.ctx.call("ske_bf_madd", f, _ptr(buf), _ptr(offs), n, _ptr(out), SKE_MEM_HOST)
        return out

    def bf_mexists_packed(self, key, buf: np.ndarray, offs: np.ndarray) -> np.ndarray:
        """BF.MEXISTS over a packed batch; missing key -> zeros."""
        key = encode(key)
        n = len(offs) - 1
        out = np.zeros(n, np.uint8)
        if not self.keys.expect(key, "bf") or n == 0:
            return out
        self.ctx.call("ske_bf_mexists", self.keys.fid[key], _ptr(buf), _ptr(offs), n, _ptr(out),
                      SKE_MEM_HOST)
        return out

    def _bf_madd_reply(self, key: bytes, items: Sequence) -> list:
        buf, offs = pack(items)
        res = self.bf_madd_packed(key, buf, offs)
        return [ResponseError("ERR non scaling filter is full") if r == -2 else int(r) for r in res]

    def bf_info(self, key) -> dict:
        key = encode(key)
        if not self.keys.expect(key, "bf"):
            raise ResponseError("ERR not found")
        info = BfInfo()
        self.ctx.call("ske_bf_info", self.keys.fid[key], C.byref(info))
        return {"Capacity": info.capacity, "Size": info.size_bytes,
                "Number of filters": info.nfilters, "Number of items inserted": info.inserted,
                "Expansion rate": None if info.nonscaling else info.expansion}

    def bf_links(self, key) -> list[dict]:
        """BF.DEBUG-like view: one dict per link (bloom_init geometry)."""
        key = encode(key)
        if not self.keys.expect(key, "bf"):
            raise ResponseError("ERR not found")
        f = self.keys.fid[key]
        info = BfInfo()
        self.ctx.call("ske_bf_info", f, C.byref(info))
        out = []
        for i in range(info.nfilters):
            L = BfLink()
            self.ctx.call("ske_bf_link_info", f, i, C.byref(L))
            out.append(dict(entries=L.entries, bytes=L.bytes, bits=L.bits, size=L.size,
                            error=L.error, bpe=L.bpe, hashes=L.hashes))
        return out

    def bf_link_bits(self, key, link: int) -> np.ndarray:
        """Raw bit array of one link (BF.SCANDUMP data chunk layout)."""
        key = encode(key)
        if not self.keys.expect(key, "bf"):
            raise ResponseError("ERR not found")
        links = self.bf_links(key)
        out = np.zeros(links[link]["bytes"], np.uint8)
        self.ctx.call("ske_bf_export_link", self.keys.fid[key], link, _ptr(out), out.size)
        return out

    # ---- BF.SCANDUMP / BF.LOADCHUNK (RedisBloom rebloom.c BFScanDump /
    # BFLoadChunk, src/sb.c SBChain_GetEncodedHeader / GetEncodedChunk /
    # LoadEncodedChunk; [recall], unconfirmed on a Redis box).  Iterator 0
    # returns the header chunk with iterator 1; iterator i > 0 returns the bytes
    # at offset i - 1 of the links' bit arrays laid end to end, at most one link
    # and MAX_SCANDUMP_SIZE bytes per chunk, with the next iterator i + len;
    # past the end it returns (0, empty).  LOADCHUNK takes the iterator that
    # SCANDUMP returned with the chunk (offset = iter - 1 - len).
    MAX_SCANDUMP_SIZE = 10 * 1024 * 1024

    def bf_scandump(self, key, it: int) -> tuple[int, bytes]:
        key = encode(key)
        if not self.keys.expect(key, "bf"):
            raise ResponseError("ERR not found")
        it = int(it)
        links = self.bf_links(key)
        if it == 0:
            info = BfInfo()
            self.ctx.call("ske_bf_info", self.keys.fid[key], C.byref(info))
            hdr = formats.bf_dump_header(info.inserted, links, info.expansion, bool(info.nonscaling))
            return 1, hdr
        off = it - 1
        for i, L in enumerate(links):
            if off < L["bytes"]:
                n = min(L["bytes"] - off, self.MAX_SCANDUMP_SIZE)
                bits = self.bf_link_bits(key, i)
                return it + n, bits[off:off + n].tobytes()
            off -= L["bytes"]
        return 0, b""

    def bf_loadchunk(self, key, it: int, data: bytes) -> bool:
        key = encode(key)
        it, data = int(it), bytes(encode(data))
        if it == 1:
            try:
                h = formats.bf_parse_header(data)
            except Exception:
                raise ResponseError("ERR received bad data")
            if self.keys.type_of(key) is not None:
                raise ResponseError("ERR item exists")
            if h["options"] & formats.BLOOM_OPT_FORCE64 == 0 or not h["links"]:
                raise ResponseError("ERR received bad data")
            arr = (BfLink * len(h["links"]))()
            for i, L in enumerate(h["links"]):
                arr[i].entries, arr[i].bytes, arr[i].bits = L["entries"], L["bytes"], L["bits"]
                arr[i].size, arr[i].error, arr[i].bpe, arr[i].hashes = (
                    L["size"], L["error"], L["bpe"], L["hashes"])
            fid = self.keys.new_fid(key)
            try:
                self.ctx.call("ske_bf_load_header", fid, arr, len(h["links"]), h["size"],
                              h["growth"], 1 if h["nonscaling"] else 0)
            except SketchLibError as e:
                self.keys.drop(key)
                raise ResponseError("ERR received bad data") from e
            return True
        if not self.keys.expect(key, "bf"):
            raise ResponseError("ERR not found")
        off = it - 1 - len(data)
        if off < 0:
            raise ResponseError("ERR invalid offset - no link found")
        for i, L in enumerate(self.bf_links(key)):
            if off < L["bytes"]:
                if off + len(data) > L["bytes"]:
                    raise ResponseError("ERR invalid chunk - Too big for current filter")
                buf = np.frombuffer(data, np.uint8)
                self.ctx.call("ske_bf_link_write", self.keys.fid[key], i, off, _ptr(buf), buf.size)
                return True
            off -= L["bytes"]
        raise ResponseError("ERR invalid offset - no link found")

    def bf(self) -> "BloomCommands":
        return BloomCommands(self)

    # ------------------------------------------------------------ HLL
    def _hll_slots_for_add(self, keys: Sequence[bytes]):
        """slot per key, creating missing keys; returns (slots, created_flags)."""
        slots, created = [], []
        for k in keys:
            if self.keys.expect(k, "hll"):
                slots.append(self.keys.slot[k])
                created.append(False)
            else:
                slots.append(self.keys.new_slot(k))
                created.append(True)
        return slots, created

    def pfadd_calls(self, calls: Sequence[tuple]) -> list[int]:
        """Several PFADD calls executed as one device batch with Redis's
        sequential replies: call c replies 1 if it created its key or any of
        its elements raised a register given all elements before it."""
        keys = [encode(c[0]) for c in calls]
        for k in keys:  # type check before any side effect
            self.keys.expect(k, "hll")
        created = []
        slots = []
        seen_new = set()
        for k in keys:
            if k in self.keys.slot:
                slots.append(self.keys.slot[k])
                created.append(False)
            else:
                slots.append(self.keys.new_slot(k))
                created.append(k not in seen_new)
                seen_new.add(k)
        elems, owner = [], []
        for ci, c in enumerate(calls):
            for v in c[1:]:
                elems.append(v)
                owner.append(ci)
        replies = [1 if cr else 0 for cr in created]
        if elems:
            buf, offs = pack(elems)
            slot_arr = np.asarray([slots[o] for o in owner], dtype=np.uint32)
            changed = np.zeros(len(elems), np.uint8)
            self.ctx.call("ske_hll_pfadd", _ptr(slot_arr), _ptr(buf), _ptr(offs), len(elems),
                          _ptr(changed), SKE_MEM_HOST)
            any_changed = np.zeros(len(calls), np.uint8)
            np.maximum.at(any_changed, np.asarray(owner, dtype=np.int64), changed)
            replies = [1 if (replies[i] or any_changed[i]) else 0 for i in range(len(calls))]
        return replies

    def pfadd(self, name, *values) -> int:
        return self.pfadd_calls([(name, *values)])[0]

    def pfadd_packed(self, slots: np.ndarray, buf: np.ndarray, offs: np.ndarray,
                     changed: bool = False) -> np.ndarray | None:
        """PFADD of (slot, element) pairs already resolved to slots."""
        n = len(offs) - 1
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        out = np.zeros(n, np.uint8) if changed else None
        if n:
            self.ctx.call("ske_hll_pfadd", _ptr(slots), _ptr(buf), _ptr(offs), n, _ptr(out),
                          SKE_MEM_HOST)
        return out

    def _count_slots(self, names) -> list[int]:
        slots = []
        for n in names:
            k = encode(n)
            if self.keys.expect(k, "hll"):
                slots.append(self.keys.slot[k])
        return slots

    def pfcount(self, *sources) -> int:
        if not sources:
            raise ResponseError("ERR wrong number of arguments for 'pfcount' command")
        slots = self._count_slots(sources)
        if not slots:
            return 0
        arr = np.asarray(slots, dtype=np.uint32)
        out = np.zeros(1, np.uint64)
        self.ctx.call("ske_hll_pfcount", _ptr(arr), len(slots), _ptr(out))
        return int(out[0])

    def pfcount_each(self, keys: Sequence) -> np.ndarray:
        """PFCOUNT of every key separately, one device launch (K2)."""
        slots = []
        present = []
        for n in keys:
            k = encode(n)
            ok = self.keys.expect(k, "hll")
            present.append(ok)
            slots.append(self.keys.slot[k] if ok else 0)
        out = np.zeros(len(slots), np.uint64)
        idx = np.flatnonzero(present)
        if idx.size:
            arr = np.asarray([slots[i] for i in idx], dtype=np.uint32)
            sub = np.zeros(idx.size, np.uint64)
            self.ctx.call("ske_hll_pfcount_each", _ptr(arr), arr.size, _ptr(sub), SKE_MEM_HOST)
            out[idx] = sub
        return out

    def pfcount_groups(self, groups: Sequence[Sequence]) -> np.ndarray:
        """PFCOUNT(k1 k2 ...) for many key groups in one launch (unions)."""
        slots, goffs = [], [0]
        for g in groups:
            slots.extend(self._count_slots(g))
            goffs.append(len(slots))
        out = np.zeros(len(groups), np.uint64)
        if groups:
            s = np.asarray(slots if slots else [0], dtype=np.uint32)
            go = np.asarray(goffs, dtype=np.uint32)
            self.ctx.call("ske_hll_pfcount_groups", _ptr(s), _ptr(go), len(groups), _ptr(out),
                          SKE_MEM_HOST)
        return out

    def pfmerge(self, dest, *sources) -> bool:
        d = encode(dest)
        src = [encode(s) for s in sources]
        for k in src:
            self.keys.expect(k, "hll")
        if not self.keys.expect(d, "hll"):
            self.keys.new_slot(d)
        slots = np.asarray([self.keys.slot[k] for k in src if k in self.keys.slot], dtype=np.uint32)
        self.ctx.call("ske_hll_pfmerge", self.keys.slot[d], _ptr(slots), slots.size)
        return True

    def hll_registers(self, name) -> np.ndarray:
        """Raw registers (Redis HLL_RAW view, one byte per register)."""
        k = encode(name)
        out = np.zeros(HLL_REGISTERS, np.uint8)
        if self.keys.expect(k, "hll"):
            self.ctx.call("ske_hll_export_raw", self.keys.slot[k], _ptr(out))
        return out

    def hll_dense(self, name) -> bytes:
        """The 12288-byte HLL_DENSE register payload of the key."""
        k = encode(name)
        if not self.keys.expect(k, "hll"):
            raise ResponseError("ERR no such key")
        out = np.zeros(HLL_DENSE_BYTES, np.uint8)
        self.ctx.call("ske_hll_export_dense", self.keys.slot[k], _ptr(out))
        return out.tobytes()

    def hll_load_registers(self, name, regs: np.ndarray) -> None:
        k = encode(name)
        if not self.keys.expect(k, "hll"):
            self.keys.new_slot(k)
        r = np.ascontiguousarray(regs, dtype=np.uint8)
        if r.shape != (HLL_REGISTERS,):
            raise DataError("expected 16384 registers")
        self.ctx.call("ske_hll_import_raw", self.keys.slot[k], _ptr(r))

    def dump_hll(self, name) -> bytes | None:
        """The key as Redis stores it (GET of an HLL key): "HYLL" header +
        canonical sparse or dense payload (formats.encode_hll)."""
        k = encode(name)
        if not self.keys.expect(k, "hll"):
            return None
        return formats.encode_hll(self.hll_registers(k))

    def load_hll(self, name, value: bytes) -> None:
        """SET of a Redis HLL string (dense or sparse) into a key."""
        regs = formats.decode_hll(bytes(value))
        k = encode(name)
        if k in self.keys.kind and self.keys.kind[k] != "hll":
            self.keys.drop(k)  # SET replaces a key of any type
        self.hll_load_registers(k, regs)

    def key_slot(self, name, create: bool = True) -> int:
        """Slot of an HLL key (creating it when asked) for batched calls."""
        k = encode(name)
        if self.keys.expect(k, "hll"):
            return self.keys.slot[k]
        if not create:
            raise ResponseError("ERR no such key")
        return self.keys.new_slot(k)

    # ------------------------------------------------------------ fused hot path
    def swipes(self, bf_key, hll_keys, items=None, *, packed=None) -> np.ndarray:
        """Batched attendance_processor.py:109-129: for every event
        ``valid = BF.EXISTS bf_key id``; if valid ``PFADD hll_key id``.

        ``hll_keys``: one key for the whole batch or one key per item.
        ``items``: ids (encoded as redis-py does) or ``packed=(buf, offs)``.
        Returns the per-event validity (bool array).  HLL keys that receive
        no valid event are not created, exactly as in the per-event loop."""
        if packed is None:
            buf, offs = pack(items)
        else:
            buf, offs = packed
            buf = np.ascontiguousarray(buf, np.uint8)
            offs = np.ascontiguousarray(offs, np.uint32)
        n = len(offs) - 1
        bkey = encode(bf_key)
        has_bf = self.keys.expect(bkey, "bf")
        if n == 0:
            return np.zeros(0, bool)
        if isinstance(hll_keys, (str, bytes, int, float)):
            key_list = [encode(hll_keys)]
            slot_idx = np.zeros(n, np.int64)
        else:
            hk = [encode(k) for k in hll_keys]
            if len(hk) != n:
                raise DataError("hll_keys must be one key or one key per item")
            uniq = {}
            slot_idx = np.fromiter((uniq.setdefault(k, len(uniq)) for k in hk), np.int64, count=n)
            key_list = list(uniq)
        for k in key_list:
            self.keys.expect(k, "hll")
        tentative = [k for k in key_list if k not in self.keys.slot]
        key_slots = np.asarray([self.keys.slot[k] if k in self.keys.slot else self.keys.new_slot(k)
                                for k in key_list], dtype=np.uint32)
        slots = key_slots[slot_idx]
        valid = np.zeros(n, np.uint8)
        if has_bf:
            self.ctx.call("ske_swipes", self.keys.fid[bkey], _ptr(slots), _ptr(buf), _ptr(offs), n,
                          _ptr(valid), SKE_MEM_HOST)
        if tentative:
            hit = np.zeros(len(key_list), bool)
            hit[np.unique(slot_idx[valid.astype(bool)])] = True
            for k in tentative:
                if not hit[key_list.index(k)]:
                    self.keys.release_unused_slot(k)
        return valid.astype(bool)

    def swipes_slots(self, bf_key, slots: np.ndarray, buf: np.ndarray, offs: np.ndarray) -> np.ndarray:
        """``swipes`` with keys already resolved to slots (see ``key_slot``)."""
        n = len(offs) - 1
        valid = np.zeros(n, np.uint8)
        bkey = encode(bf_key)
        if n and self.keys.expect(bkey, "bf"):
            s = np.ascontiguousarray(slots, dtype=np.uint32)
            self.ctx.call("ske_swipes", self.keys.fid[bkey], _ptr(s), _ptr(buf), _ptr(offs), n,
                          _ptr(valid), SKE_MEM_HOST)
        return valid.astype(bool)

    def swipes_fixed(self, bf_key, slots: np.ndarray, ids: np.ndarray) -> np.ndarray:
        """``swipes_slots`` for ids of one fixed width: ``ids`` is a [n, width]
        uint8 array of the ids' bytes (e.g. 8-digit student ids as redis-py
        encodes them).  Through ske_swipes_fixed_bits: no offsets cross the
        host link and the answers come back 1 bit per swipe, in chunks that
        overlap the copies with the kernels."""
        ids = np.ascontiguousarray(ids, dtype=np.uint8)
        if ids.ndim != 2:
            raise ValueError("ids must be a [n, width] uint8 array")
        n, width = ids.shape
        bits = np.zeros((n + 7) // 8, np.uint8)
        bkey = encode(bf_key)
        if n and width and self.keys.expect(bkey, "bf"):
            s = np.ascontiguousarray(slots, dtype=np.uint32)
            if s.shape != (n,):
                raise ValueError("one slot per id")
            self.ctx.call("ske_swipes_fixed_bits", self.keys.fid[bkey], _ptr(s), _ptr(ids), width, n,
                          _ptr(bits), SKE_MEM_HOST)
        return np.unpackbits(bits, count=n, bitorder="little").astype(bool)

    # ------------------------------------------------------------ ingest (§8f row 3)
    def ingest(self, bf_key, messages: Sequence, hll_key_prefix: str = "hll:unique:",
               key_form: str = "readme") -> tuple[np.ndarray, np.ndarray]:
        """The processor loop of attendance_processor.py:100-137 over raw
        message payloads: decode (json.loads, :103-106), BF.EXISTS of the
        student id (:109-113) and, if valid, PFADD into the lecture key (:128;
        README.md:105-106 form ``<prefix><lecture_id>:<YYYY-MM-DD>`` with the
        UTC day, or ``key_form="code"``: ``<prefix><lecture_id>``).

        Messages are decoded on the device (sketch_ingest.hip); those outside
        its fast JSON / ISO-8601 path go through Python's json / datetime here,
        so every message gets exactly the reference's treatment.  Returns
        ``(valid, status)``: per message the BF.EXISTS answer and 0 decoded on
        the device, 1 decoded on the host, -1 not decodable (the reference's
        negative_acknowledge, :134-136)."""
        n = len(messages)
        try:
            joined = b"".join(messages)
            raw = messages
        except TypeError:  # str payloads: as .decode() would see them
            raw = [m if isinstance(m, (bytes, bytearray, memoryview)) else str(m).encode()
                   for m in messages]
            joined = b"".join(raw)
        lens = np.fromiter(map(len, raw), np.uint32, count=n)
        moffs = np.zeros(n + 1, np.uint32)
        np.cumsum(lens, out=moffs[1:])
        return self.ingest_packed(bf_key, np.frombuffer(joined, np.uint8), moffs, hll_key_prefix,
                                  key_form)

    def ingest_packed(self, bf_key, blob: np.ndarray, moffs: np.ndarray,
                      hll_key_prefix: str = "hll:unique:", key_form: str = "readme"):
        """``ingest`` over payloads already laid end to end: message i is
        ``blob[moffs[i]:moffs[i+1]]`` (the layout a network consumer fills)."""
        import json
        from datetime import datetime, timezone
        from ._lib import IngestCols
        blob = np.ascontiguousarray(blob, np.uint8)
        moffs = np.ascontiguousarray(moffs, np.uint32)
        n = len(moffs) - 1
        valid = np.zeros(n, bool)
        status = np.zeros(n, np.int8)
        if n <= 0:
            return valid, status
        day_form = 1 if key_form == "readme" else 0
        prefix = str(hll_key_prefix)
        mv = memoryview(blob)

        class _Raw:  # message i as bytes (host-path decode only)
            def __getitem__(self, i):
                return mv[moffs[i]:moffs[i + 1]].tobytes()

        raw = _Raw()
        B = self._ingest_buffers(n, blob.size)
        if blob.size:
            self.ctx.call("ske_memcpy", C.c_void_p(B["msgs"].ptr), _ptr(blob), blob.size, 0)
        self.ctx.call("ske_memcpy", C.c_void_p(B["moffs"].ptr), _ptr(moffs), moffs.nbytes, 0)
        cols = IngestCols(*[C.c_void_p(B[k].ptr) for k in
                            ("status", "id_start", "id_len", "lec_start", "lec_len", "ts_start",
                             "ts_len", "day", "kh")])
        self.ctx.call("ske_ingest_parse", C.c_void_p(B["msgs"].ptr), C.c_void_p(B["moffs"].ptr), n,
                      day_form, C.byref(cols))
        if self._kt_state != (self.keys.slots_released, day_form, prefix):
            self.ctx.call("ske_keytab_clear")  # a freed slot may be reused: start over
            self._kt_state = (self.keys.slots_released, day_form, prefix)
        nmiss = C.c_uint64()
        self.ctx.call("ske_keytab_lookup", C.byref(cols), n, C.c_void_p(B["slot"].ptr), C.byref(nmiss))
        dev_status = B["status"].to_host(np.uint8, n)

        def key_name(data) -> bytes:
            lecture_id = data["lecture_id"]
            ts = datetime.fromisoformat(data["timestamp"])
            if key_form == "code":
                return encode(f"{prefix}{lecture_id}")
            if ts.tzinfo is not None:
                ts = ts.astimezone(timezone.utc)
            return encode(f"{prefix}{lecture_id}:{ts.date().isoformat()}")

        tentative = []
        if nmiss.value:
            # keys seen for the first time: one Python decode per new key
            slot = B["slot"].to_host(np.uint32, n)
            kh = B["kh"].to_host(np.uint64, 2 * n).reshape(n, 2)
            miss = np.nonzero((dev_status == 0) & (slot == 0xFFFFFFFF))[0]
            uk, first = np.unique(kh[miss], axis=0, return_index=True)
            new_slots = np.zeros(len(uk), np.uint32)
            for j, m in enumerate(miss[first]):
                name = key_name(json.loads(bytes(raw[m]).decode()))
                self.keys.expect(name, "hll")
                if name not in self.keys.slot:
                    tentative.append(name)
                    new_slots[j] = self.keys.new_slot(name)
                else:
                    new_slots[j] = self.keys.slot[name]
            ukc = np.ascontiguousarray(uk, np.uint64)
            self.ctx.call("ske_keytab_insert", ukc.ctypes.data_as(C.c_void_p), _ptr(new_slots), len(uk))
        bkey = encode(bf_key)
        has_bf = self.keys.expect(bkey, "bf")
        taken = C.c_uint64()
        if has_bf:
            self.ctx.call("ske_ingest_swipes", self.keys.fid[bkey], C.c_void_p(B["msgs"].ptr),
                          C.byref(cols), n, C.c_void_p(B["valid"].ptr), C.byref(taken))
            valid[:] = B["valid"].to_host(np.uint8, n).astype(bool)
        # the rest: Python's json / datetime semantics
        host = np.nonzero(dev_status != 0)[0]
        ids, keys, at = [], [], []
        for m in host:
            try:
                data = json.loads(bytes(raw[m]).decode())
                sid = encode(data["student_id"])
                name = key_name(data)
            except Exception:
                status[m] = -1
                continue
            status[m] = 1
            ids.append(sid)
            keys.append(name)
            at.append(m)
        if at:
            valid[np.asarray(at)] = self.swipes(bkey, keys, ids)
        if tentative:
            # keys created for this batch that no valid swipe reached are not
            # created (as in the per-event loop)
            hit = set()
            if has_bf:
                self.ctx.call("ske_keytab_lookup", C.byref(cols), n, C.c_void_p(B["slot"].ptr), None)
                slot = B["slot"].to_host(np.uint32, n)
                hit = set(np.unique(slot[valid & (dev_status == 0)]).tolist())
                hit |= {self.keys.slot[k] for k, m in zip(keys, at) if valid[m] and k in self.keys.slot}
            for name in tentative:
                if name in self.keys.slot and self.keys.slot[name] not in hit:
                    self.keys.release_unused_slot(name)
        return valid, status

    def _ingest_buffers(self, n: int, nbytes: int) -> dict:
        from .engine import DeviceBuffer
        B = getattr(self, "_ingest_bufs", None)
        if B is None or B["n"] < n or B["nbytes"] < nbytes:
            if B is not None:
                for k, v in B.items():
                    if k not in ("n", "nbytes"):
                        v.free()
            cn, cb = max(n, 1024), max(nbytes, 1 << 16)
            B = {"n": cn, "nbytes": cb, "msgs": DeviceBuffer(self.ctx, cb + 64),
                 "moffs": DeviceBuffer(self.ctx, (cn + 1) * 4), "status": DeviceBuffer(self.ctx, cn),
                 "day": DeviceBuffer(self.ctx, cn * 4), "kh": DeviceBuffer(self.ctx, cn * 16),
                 "slot": DeviceBuffer(self.ctx, cn * 4), "valid": DeviceBuffer(self.ctx, cn)}
            for k in ("id_start", "id_len", "lec_start", "lec_len", "ts_start", "ts_len"):
                B[k] = DeviceBuffer(self.ctx, cn * 4)
            self._ingest_bufs = B
        return B

    # ------------------------------------------------------------ command dispatch
    def execute_command(self, *args, **options):
        if not args:
            raise ResponseError("ERR empty command")
        name = args[0].decode() if isinstance(args[0], bytes) else str(args[0])
        cmd = name.upper()
        a = args[1:]

        def need(lo, hi=None):
            if len(a) < lo or (hi is not None and len(a) > hi):
                raise ResponseError(f"ERR wrong number of arguments for '{name.lower()}' command")

        if cmd == "BF.RESERVE":
            need(3)
            exp, nonscaling = None, False
            rest = list(a[3:])
            while rest:
                opt = rest.pop(0)
                opt = (opt.decode() if isinstance(opt, bytes) else str(opt)).upper()
                if opt == "EXPANSION" and rest:
                    exp = rest.pop(0)
                elif opt == "NONSCALING":
                    nonscaling = True
                else:
                    raise ResponseError("ERR syntax error")
            return self._bf_reserve(encode(a[0]), a[1], a[2], exp, nonscaling)
        if cmd == "BF.ADD":
            need(2, 2)
            r = self._bf_madd_reply(encode(a[0]), [a[1]])[0]
            if isinstance(r, ResponseError):
                raise r
            return r
        if cmd == "BF.MADD":
            need(2)
            return self._bf_madd_reply(encode(a[0]), a[1:])
        if cmd in ("BF.EXISTS", "BF.MEXISTS"):
            need(2, 2 if cmd == "BF.EXISTS" else None)
            buf, offs = pack(a[1:])
            r = [int(x) for x in self.bf_mexists_packed(a[0], buf, offs)]
            return r[0] if cmd == "BF.EXISTS" else r
        if cmd == "BF.INFO":
            need(1, 1)
            info = self.bf_info(a[0])
            flat = []
            for k, v in info.items():
                flat += [self._s(k), v]
            return flat
        if cmd == "BF.SCANDUMP":
            need(2, 2)
            it, chunk = self.bf_scandump(a[0], a[1])
            return [it, chunk]
        if cmd == "BF.LOADCHUNK":
            need(3, 3)
            self.bf_loadchunk(a[0], a[1], a[2])
            return self._ok()
        if cmd == "BF.CARD":
            need(1, 1)
            k = encode(a[0])
            return self.bf_info(k)["Number of items inserted"] if self.keys.expect(k, "bf") else 0
        if cmd == "PFADD":
            need(1)
            return self.pfadd(*a)
        if cmd == "PFCOUNT":
            need(1)
            return self.pfcount(*a)
        if cmd == "PFMERGE":
            need(1)
            self.pfmerge(*a)
            return self._ok()
        if cmd == "GET":
            need(1, 1)
            k = encode(a[0])
            if self.keys.type_of(k) == "bf":
                raise ResponseError(WRONGTYPE)
            return self.dump_hll(k)
        if cmd == "SET":
            need(2, 2)
            self.load_hll(a[0], encode(a[1]))
            return self._ok()
        if cmd in ("DEL", "UNLINK"):
            need(1)
            return self.delete(*a)
        if cmd == "EXISTS":
            need(1)
            return self.exists(*a)
        if cmd == "TYPE":
            need(1, 1)
            return self.type(a[0])
        if cmd in ("FLUSHALL", "FLUSHDB"):
            self.flushall()
            return self._ok()
        if cmd == "PING":
            return self._s("PONG")
        raise ResponseError(f"ERR unknown command '{name}'")

    def pipeline(self, transaction: bool = True, shard_hint=None) -> "Pipeline":
        return Pipeline(self)


Redis = SketchClient  # redis.Redis(host=..., port=..., decode_responses=True) drop-in


class BloomCommands:
    """``client.bf()`` surface of redis-py (redis.commands.bf.BFCommands)."""

    def __init__(self, client: SketchClient):
        self.client = client

    def create(self, key, errorRate, capacity, expansion=None, noScale=None):
        self.client._bf_reserve(encode(key), errorRate, capacity, expansion, bool(noScale))
        return True

    reserve = create

    def add(self, key, item):
        return self.client.execute_command("BF.ADD", key, item)

    def madd(self, key, *items):
        return self.client.execute_command("BF.MADD", key, *items)

    def exists(self, key, item):
        return self.client.execute_command("BF.EXISTS", key, item)

    def mexists(self, key, *items):
        return self.client.execute_command("BF.MEXISTS", key, *items)

    def info(self, key):
        return BFInfo(self.client.bf_info(key))

    def card(self, key):
        return self.client.execute_command("BF.CARD", key)


class BFInfo:
    """redis.commands.bf.info.BFInfo attribute names."""

    def __init__(self, d: dict):
        self.capacity = d["Capacity"]
        self.size = d["Size"]
        self.filterNum = d["Number of filters"]
        self.insertedNum = d["Number of items inserted"]
        self.expansionRate = d["Expansion rate"]

    def get(self, item):
        return getattr(self, item)

    def __getitem__(self, item):
        return getattr(self, item)


class Pipeline:
    """redis-py pipeline: commands are queued and executed on ``execute()``.

    Consecutive compatible commands run as ONE device batch with Redis's
    sequential replies: a run of PFADDs (any keys) becomes one exact-order
    ske_hll_pfadd; a run of BF.EXISTS/BF.MEXISTS on one key one
    ske_bf_mexists; a run of BF.ADD/BF.MADD on one key one ske_bf_madd."""

    def __init__(self, client: SketchClient):
        self.client = client
        self._cmds: list[tuple] = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.reset()

    def __len__(self):
        return len(self._cmds)

    def reset(self):
        self._cmds = []

    def execute_command(self, *args, **options):
        self._cmds.append(args)
        return self

    def pfadd(self, name, *values):
        return self.execute_command("PFADD", name, *values)

    def pfcount(self, *sources):
        return self.execute_command("PFCOUNT", *sources)

    def pfmerge(self, dest, *sources):
        return self.execute_command("PFMERGE", dest, *sources)

    def bf(self):
        p = self

        class _B:
            def add(self, key, item):
                return p.execute_command("BF.ADD", key, item)

            def madd(self, key, *items):
                return p.execute_command("BF.MADD", key, *items)

            def exists(self, key, item):
                return p.execute_command("BF.EXISTS", key, item)

            def mexists(self, key, *items):
                return p.execute_command("BF.MEXISTS", key, *items)

            def reserve(self, key, errorRate, capacity, expansion=None, noScale=None):
                args = ["BF.RESERVE", key, errorRate, capacity]
                if expansion is not None:
                    args += ["EXPANSION", expansion]
                if noScale:
                    args += ["NONSCALING"]
                return p.execute_command(*args)

            create = reserve
        return _B()

    @staticmethod
    def _name(c) -> str:
        n = c[0]
        return (n.decode() if isinstance(n, bytes) else str(n)).upper()

    def execute(self, raise_on_error: bool = True) -> list:
        cmds, self._cmds = self._cmds, []
        out: list = []
        i = 0
        cl = self.client
        while i < len(cmds):
            name = self._name(cmds[i])
            j = i + 1
            try:
                if name == "PFADD" and len(cmds[i]) >= 2:
                    while j < len(cmds) and self._name(cmds[j]) == "PFADD" and len(cmds[j]) >= 2:
                        j += 1
                    out.extend(cl.pfadd_calls([c[1:] for c in cmds[i:j]]))
                elif name in ("BF.EXISTS", "BF.MEXISTS") and len(cmds[i]) >= 3:
                    key = encode(cmds[i][1])
                    while (j < len(cmds) and self._name(cmds[j]) in ("BF.EXISTS", "BF.MEXISTS")
                           and len(cmds[j]) >= 3 and encode(cmds[j][1]) == key):
                        j += 1
                    if any(self._name(c) == "BF.EXISTS" and len(c) != 3 for c in cmds[i:j]):
                        raise ResponseError("ERR wrong number of arguments for 'bf.exists' command")
                    items = [x for c in cmds[i:j] for x in c[2:]]
                    buf, offs = pack(items)
                    res = cl.bf_mexists_packed(key, buf, offs)
                    p = 0
                    for c in cmds[i:j]:
                        m = len(c) - 2
                        r = [int(x) for x in res[p:p + m]]
                        out.append(r[0] if self._name(c) == "BF.EXISTS" else r)
                        p += m
                elif name in ("BF.ADD", "BF.MADD") and len(cmds[i]) >= 3:
                    key = encode(cmds[i][1])
                    while (j < len(cmds) and self._name(cmds[j]) in ("BF.ADD", "BF.MADD")
                           and len(cmds[j]) >= 3 and encode(cmds[j][1]) == key):
                        j += 1
                    items = [x for c in cmds[i:j] for x in c[2:]]
                    res = cl._bf_madd_reply(key, items)
                    p = 0
                    for c in cmds[i:j]:
                        m = len(c) - 2
                        out.append(res[p] if self._name(c) == "BF.ADD" else res[p:p + m])
                        p += m
                else:
                    out.append(cl.execute_command(*cmds[i]))
            except ResponseError as e:
                out.extend([e] * (j - i))
            i = j
        if raise_on_error:
            for r in out:
                if isinstance(r, ResponseError):
                    raise r
        return out
