"""Pin the CPU oracle to published known answers before trusting it.

- MurmurHash64A: SMHasher's VerificationTest value for MurmurHash64A is
  0x1F0D3804 (the routine Redis hyperloglog.c and RedisBloom MurmurHash2.c
  both carry).
- HyperLogLog: the Redis command documentation examples
  (PFADD hll a b c d e f g -> PFCOUNT 7; foo bar zap + repeats -> 3;
  PFCOUNT hll some-other-hll{1,2,3} -> 6; PFMERGE {foo,bar,zap,a} u
  {a,b,c,foo} -> 6).
- RedisBloom geometry: the table of SURVEY.md §8a-6 (restated from
  bloom_init / SB_NewChain; not confirmed on a Redis box -- "unpinned").
"""
import numpy as np


def test_smhasher_verification(orc):
    assert orc.smhasher_verification() == 0x1F0D3804


def test_pfcount_docs_examples(orc):
    h = orc.HLL()
    assert h.add(*[c.encode() for c in "abcdefg"]) == 1
    assert h.count() == 7

    h = orc.HLL()
    h.add(b"foo", b"bar", b"zap")
    h.add(b"zap", b"zap", b"zap")
    h.add(b"foo", b"bar")
    assert h.count() == 3
    other = orc.HLL()
    other.add(b"1", b"2", b"3")
    u = orc.HLL(h.regs)
    u.merge(other)
    assert u.count() == 6


def test_pfmerge_docs_example(orc):
    a, b = orc.HLL(), orc.HLL()
    a.add(b"foo", b"bar", b"zap", b"a")
    b.add(b"a", b"b", b"c", b"foo")
    a.merge(b)
    assert a.count() == 6


def test_pfadd_reply_semantics(orc):
    h = orc.HLL()
    assert h.add(b"x") == 1
    assert h.add(b"x") == 0  # no register changed


def test_decimal_id_sanity(orc):
    h = orc.HLL()
    h.add(*[str(i).encode() for i in range(10000, 11000)])
    assert h.count() == 1001
    h = orc.HLL()
    h.add(*[str(i).encode() for i in range(10000, 110000)])
    assert h.count() == 100435


def test_estimator_edges(orc):
    histo = np.zeros(64, np.int32)
    histo[0] = 16384
    assert orc.hll_estimate(histo) == 0  # sigma(1) = inf -> 0
    assert orc.lib().orc_hll_tau(0.0) == 0.0 and orc.lib().orc_hll_tau(1.0) == 0.0


def test_bloom_geometry_table(orc):
    c = orc.Chain(100000, 0.01)
    assert c.link_info(0) == dict(entries=100000, bytes=137848, bits=1102784, hashes=8, size=0,
                                  error=0.005)
    c = orc.Chain(10_000_000, 0.001)
    li = c.link_info(0)
    assert (li["bytes"], li["bits"], li["hashes"]) == (19775360, 158202880, 11)


def test_default_chain_growth(orc):
    # BF.ADD auto-create (100 / 0.01 / x2) and 1000 distinct ids -> 4 links
    c = orc.Chain(100, 0.01)
    for i in range(10000, 11000):
        c.add(str(i).encode())
    assert c.nlinks == 4
    got = [(c.link_info(i)["entries"], c.link_info(i)["bytes"], c.link_info(i)["hashes"])
           for i in range(4)]
    assert got == [(100, 144, 8), (200, 312, 9), (400, 696, 10), (800, 1536, 11)]


def test_nonscaling_full(orc):
    c = orc.Chain(10, 0.01, nonscaling=True)
    res = [c.add(str(i).encode()) for i in range(100, 140)]
    assert res.count(-2) > 0
    assert c.size == 10


def test_hll_string_decode(orc):
    # new key: "HYLL" sparse, one XZERO opcode covering 16384 registers
    s = b"HYLL" + bytes([1, 0, 0, 0]) + bytes(8) + bytes([0x7F, 0xFF])
    regs = orc.hll_decode_string(s)
    assert regs is not None and not regs.any()
    # VAL opcode: value 3, run 2 at the start, then XZERO for the rest
    rest = 16384 - 2 - 1
    s = b"HYLL" + bytes([1, 0, 0, 0]) + bytes(8) + bytes([0x80 | (2 << 2) | 1,
                                                           0x40 | (rest >> 8), rest & 0xFF])
    regs = orc.hll_decode_string(s)
    assert regs[:2].tolist() == [3, 3] and not regs[2:].any()
    # dense round trip
    h = orc.HLL()
    h.add(*[str(i).encode() for i in range(5000)])
    s = b"HYLL" + bytes([0, 0, 0, 0]) + bytes(8) + h.dense()
    assert np.array_equal(orc.hll_decode_string(s), h.regs)
    assert orc.hll_decode_string(b"HYLL" + bytes([1, 0, 0, 0]) + bytes(8) + bytes([0x00])) is None


def test_process_swipes_threads_identical(orc):
    """The multi-threaded CPU baseline (orc_process_swipes_mt, bench.py's
    cpu_baseline) gives the sequential loop's answers, counts and registers."""
    rng = np.random.default_rng(3)
    members = rng.choice(np.arange(10**5, 10**6), 3000, replace=False)
    chain = orc.Chain(5000, 0.01)
    chain.madd_packed(*orc.pack([str(int(x)).encode() for x in members]))
    ids = np.where(rng.random(20000) < 0.9, rng.choice(members, 20000),
                   rng.integers(10**6, 2 * 10**6, 20000))
    buf, offs = orc.pack([str(int(x)).encode() for x in ids])
    slot = rng.integers(0, 37, 20000).astype(np.uint32)
    want = np.zeros((37, 16384), np.uint8)
    v1, n1, p1 = orc.process_swipes(chain, want, slot, buf, offs)
    for threads in (2, 5, 16):
        got = np.zeros_like(want)
        v2, n2, p2 = orc.process_swipes(chain, got, slot, buf, offs, threads=threads)
        assert np.array_equal(v1, v2) and (n1, p1) == (n2, p2)
        assert np.array_equal(want, got)
