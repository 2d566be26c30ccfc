"""The oracle reproduces every committed golden vector (regression pin)."""
import ctypes as C
import hashlib

import numpy as np


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def test_murmur_vectors(orc, golden):
    for data_hex, seed, want in golden["murmur64a"]:
        assert orc.murmur64a(bytes.fromhex(data_hex), int(seed)) == int(want)


def test_patlen_vectors(orc, golden):
    for x, idx, cnt in golden["hll_patlen"]:
        b = str(x).encode()
        r = C.c_long()
        assert orc.lib().orc_hll_patlen(b, len(b), C.byref(r)) == cnt
        assert r.value == idx


def test_hll_sets(orc, golden, golden_arrays):
    for name, want in golden["hll_sets"].items():
        regs = golden_arrays[f"hll_{name}"]
        assert sha(regs) == want["regs_sha256"]
        assert orc.hll_count_regs(regs) == want["count"]
        assert sha(orc.HLL(regs).dense()) == want["dense_sha256"]


def test_hll_sets_rebuilt(orc, golden):
    h = orc.HLL()
    h.add(*[str(i).encode() for i in range(10000, 11000)])
    assert sha(h.regs) == golden["hll_sets"]["ints_10000_10999"]["regs_sha256"]


def test_estimator_vectors(orc, golden):
    for e in golden["hll_estimate"]:
        assert orc.hll_estimate(np.array(e["histo"], np.int32)) == e["count"]


def test_bloom_geometry(orc, golden):
    for g in golden["bloom_geometry"]:
        li = orc.Chain(g["capacity"], g["error"] * 2).link_info(0)  # SB_NewChain halves it
        for k in ("entries", "bytes", "bits", "hashes"):
            assert li[k] == g[k], (g, li)


def test_bloom_reserved(orc, golden, golden_arrays):
    g = golden["bloom_reserved_1000"]
    c = orc.Chain(1000, 0.01)
    assert [c.add(x.encode()) for x in g["ids"]] == g["replies"]
    assert c.size == g["size"]
    assert sha(c.link_bits(0)) == g["bits_sha256"]
    assert np.array_equal(c.link_bits(0), golden_arrays["reserved_1000_link0"])
    probe = [str(x).encode() for x in range(g["probe_lo"], g["probe_hi"])]
    assert [c.exists(x) for x in probe] == g["exists"]


def test_bloom_default_chain(orc, golden):
    g = golden["bloom_default_chain"]
    c = orc.Chain(100, 0.01)
    assert [c.add(x.encode()) for x in golden["bloom_reserved_1000"]["ids"]] == g["replies"]
    assert c.size == g["size"]
    assert [c.link_info(i) for i in range(c.nlinks)] == g["links"]
    assert [sha(c.link_bits(i)) for i in range(c.nlinks)] == g["bits_sha256"]
