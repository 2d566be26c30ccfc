"""Redis HLL string formats (dense / sparse) and the RedisBloom dump header:
round trips, and cross-checks against the oracle's independent decoder."""
import numpy as np
import pytest


def _regs(orc, n, seed):
    rng = np.random.default_rng(seed)
    h = orc.HLL()
    h.add(*[str(int(x)).encode() for x in rng.integers(0, 10**9, n)])
    return h.regs


@pytest.mark.parametrize("n", [0, 1, 5, 100, 2000, 20000, 300000])
def test_hll_string_round_trip(pkg, orc, n):
    from rtsas_amd import formats
    regs = _regs(orc, n, n)
    s = formats.encode_hll(regs)
    assert s[:4] == b"HYLL"
    assert np.array_equal(formats.decode_hll(s), regs)
    assert np.array_equal(orc.hll_decode_string(s), regs)      # independent decoder
    if n <= 100:
        assert s[4] == 1                                         # stays sparse when small
    dense = formats.encode_hll(regs, sparse_max_bytes=0)
    assert dense[4] == 0 and len(dense) == 16 + 12288
    assert dense[16:] == orc.HLL(regs).dense()                   # HLL_DENSE_SET_REGISTER


def test_new_key_and_cache(pkg):
    from rtsas_amd import formats
    s = formats.encode_hll(np.zeros(16384, np.uint8), card=0)
    assert s == b"HYLL\x01\x00\x00\x00" + bytes(8) + b"\x7f\xff"  # createHLLObject
    assert formats.cached_card(s) == 0
    s2 = formats.encode_hll(np.zeros(16384, np.uint8))
    assert formats.cached_card(s2) is None


def test_sparse_promotion_rule(pkg):
    from rtsas_amd import formats
    regs = np.zeros(16384, np.uint8)
    regs[5] = 33                                                 # > 32: dense only
    assert formats.encode_hll(regs)[4] == 0


def test_corrupted_strings(pkg):
    from rtsas_amd import formats
    with pytest.raises(pkg.ResponseError):
        formats.decode_hll(b"HYLL\x01\x00\x00\x00" + bytes(8) + b"\x00")    # covers 1 register
    with pytest.raises(pkg.ResponseError):
        formats.decode_hll(b"HYLL\x00\x00\x00\x00" + bytes(8) + bytes(100))  # short dense
    with pytest.raises(pkg.ResponseError):
        formats.decode_hll(b"NOPE" + bytes(20))


def test_bf_dump_header_round_trip(pkg, orc):
    from rtsas_amd import formats
    c = orc.Chain(100, 0.01)
    for i in range(1000):
        c.add(str(i).encode())
    links = [c.link_info(i) for i in range(c.nlinks)]
    for L in links:
        L["bpe"] = 0.0
    h = formats.bf_dump_header(c.size, links, 2, False)
    p = formats.bf_parse_header(h)
    assert p["size"] == c.size and p["growth"] == 2 and not p["nonscaling"]
    assert [(l["bytes"], l["entries"], l["hashes"]) for l in p["links"]] == \
        [(l["bytes"], l["entries"], l["hashes"]) for l in links]
