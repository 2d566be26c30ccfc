"""redis-py argument encoding (Encoder.encode) and the packed-item layout."""
import numpy as np
import pytest


def test_encode_rules(pkg):
    enc = pkg.encode
    assert enc(12345) == b"12345"            # data_generator.py:113 ints
    assert enc(-7) == b"-7"
    assert enc(0.01) == b"0.01"              # BF.RESERVE error rate (attendance_processor.py:86)
    assert enc("S123456") == b"S123456"      # README.md:93 string ids
    assert enc("é") == "é".encode("utf-8")
    assert enc(b"\x00\xff") == b"\x00\xff"
    assert enc(memoryview(b"ab")) == b"ab"
    assert enc(np.int64(42)) == b"42"
    with pytest.raises(pkg.DataError):
        enc(True)
    with pytest.raises(pkg.DataError):
        enc(None)
    with pytest.raises(pkg.DataError):
        enc([1])


def test_pack_layout(pkg):
    buf, offs = pkg.pack([1, "ab", b"", 99999])
    assert offs.tolist() == [0, 1, 3, 3, 8]
    assert bytes(buf) == b"1ab99999"
    buf, offs = pkg.pack([])
    assert offs.tolist() == [0] and buf.size == 0


def test_pack_ints_matches_pack(pkg):
    rng = np.random.default_rng(0)
    vals = np.concatenate([
        np.array([0, 1, 9, 10, 99, 100, 999, 10**9, 10**18, 2**63 - 1, 2**64 - 1], dtype=np.uint64),
        rng.integers(0, 2**63, 500, dtype=np.uint64),
        rng.integers(0, 10**7, 500).astype(np.uint64)])
    b1, o1 = pkg.pack_ints(vals)
    b2, o2 = pkg.pack([int(v) for v in vals])
    assert np.array_equal(o1, o2) and np.array_equal(b1, b2)
    b, o = pkg.pack_ints(np.zeros(0, np.uint64))
    assert b.size == 0 and o.tolist() == [0]


def test_keyhash_matches_oracle(orc):
    from rtsas_amd.keyhash import murmur64a
    rng = np.random.default_rng(1)
    for n in list(range(0, 30)) + [64, 100]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, 0xADC83B19, 2**64 - 1):
            assert murmur64a(d, seed) == orc.murmur64a(d, seed)


def test_redis_glob_dialect(pkg):
    """SCAN MATCH follows Redis' stringmatchlen (redis src/util.c, restated in
    client.redis_glob), not Python's fnmatch: '^' negates a class, backslash
    escapes, reversed ranges are swapped.  No Redis in this image: the cases
    are the rule read from the source -- parity unpinned."""
    from rtsas_amd.client import redis_glob as g
    assert g(b"[^a]*", b"bcd") and not g(b"[^a]*", b"abc")
    assert g(b"h[!e]llo", b"h!llo") and g(b"h[!e]llo", b"hello") and not g(b"h[!e]llo", b"hallo")  # "!" is a member
    assert g(b"foo\\*", b"foo*") and not g(b"foo\\*", b"foox")
    assert g(b"h[e-a]llo", b"hallo") and g(b"h[a-e]llo", b"hello") and not g(b"h[^e]llo", b"hello")
    assert g(b"h[\\]]llo", b"h]llo")
    assert g(b"a*c", b"abbbc") and g(b"**b", b"ab") and g(b"a?c", b"abc") and not g(b"a?c", b"ac")
    assert g(b"hll:unique:L1:????-??-??", b"hll:unique:L1:2025-03-19")
    assert not g(b"hll:unique:L1:????-??-??", b"hll:unique:L1:x:2025-03-19")
    assert not g(b"*", b"")  # stringmatchlen itself; SCAN / KEYS bypass a bare '*'


def test_glob_escape_stems(pkg):
    """processor.glob_escape (the SCAN fallback of get_attendance_stats):
    a lecture stem holding glob specials matches exactly its own day keys."""
    from rtsas_amd.client import redis_glob as g
    from rtsas_amd.processor import glob_escape
    day = ":" + "[0-9]" * 4 + "-" + "[0-9]" * 2 + "-" + "[0-9]" * 2
    for stem in ["hll:unique:A^B", "hll:unique:a]b", "hll:unique:a\\b", "hll:unique:[x]*?", "hll:unique:^",
                 "hll:unique:]", "hll:unique:\\", "hll:unique:plain"]:
        pat = (glob_escape(stem) + day).encode()
        assert g(pat, (stem + ":2025-03-19").encode()), stem
        assert not g(pat, (stem + "x:2025-03-19").encode()), stem
        assert not g(pat, (stem[:-1] + "Q:2025-03-19").encode()), stem
        assert not g(pat, (stem + ":2025-03-19:x").encode()), stem
