"""HIP path (through the C-ABI) vs the CPU oracle -- bit-exact.

Every comparison is exact: Bloom answers, Bloom bit arrays, per-item BF.ADD
replies, HLL register arrays, PFADD replies and PFCOUNT values.  Inputs are
seeded; sizes are ones the oracle finishes in seconds.  Parity is against the
oracle (a restatement of Redis / RedisBloom pinned by published KATs); parity
against a live Redis is not available in this environment.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rand_items(rng, n, maxlen=64, minlen=0):
    lens = rng.integers(minlen, maxlen + 1, n)
    return [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]


# ------------------------------------------------------------------ Bloom
def test_mexists_random_bytes_vs_oracle(client, orc):
    """Murmur + probe arithmetic on ragged byte strings (0..64 B, all
    alignments) through BF.MEXISTS."""
    rng = np.random.default_rng(1)
    members = _rand_items(rng, 3000, 64)
    chain = orc.Chain(2000, 0.02)
    client.execute_command("BF.RESERVE", "k", 0.02, 2000)
    client.execute_command("BF.MADD", "k", *members[:1500])
    for m in members[:1500]:
        chain.add(m)
    probe = members + _rand_items(rng, 5000, 64)
    got = client.execute_command("BF.MEXISTS", "k", *probe)
    want = [chain.exists(p) for p in probe]
    assert got == want


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("pb", [1, 2, 4, 8])
def test_mexists_variants(client, orc, variant, pb):
    client.ctx.call("ske_set_option", b"variant", variant)
    client.ctx.call("ske_set_option", b"tile", pb)
    rng = np.random.default_rng(2)
    ids = rng.choice(np.arange(10**6, 10**7), 30000, replace=False)
    client.execute_command("BF.RESERVE", "bf", 0.01, 20000)
    client.bf_madd_packed("bf", *client_pack(ids[:20000]))
    chain = orc.Chain(20000, 0.01)
    buf, offs = client_pack(ids[:20000])
    chain.madd_packed(buf, offs)
    buf, offs = client_pack(ids)
    got = client.bf_mexists_packed("bf", buf, offs)
    want, _ = chain.mexists_packed(buf, offs)
    assert np.array_equal(got, want)


def client_pack(ids):
    import rtsas_amd
    return rtsas_amd.pack_ints(ids)


def test_madd_reserved_matches_golden(client, orc, golden, golden_arrays):
    g = golden["bloom_reserved_1000"]
    client.execute_command("BF.RESERVE", "bf:students", 0.01, 1000)
    assert client.execute_command("BF.MADD", "bf:students", *g["ids"]) == g["replies"]
    bits = client.bf_link_bits("bf:students", 0)
    assert np.array_equal(bits, golden_arrays["reserved_1000_link0"])
    probe = [str(x) for x in range(g["probe_lo"], g["probe_hi"])]
    assert client.execute_command("BF.MEXISTS", "bf:students", *probe) == g["exists"]
    assert client.bf_info("bf:students")["Number of items inserted"] == g["size"]


def test_madd_default_chain_growth(client, golden, golden_arrays):
    """BF.ADD auto-create + growth to 4 links, order-exact replies (the
    reference's data_generator.py:57-63 flow)."""
    g = golden["bloom_default_chain"]
    ids = golden["bloom_reserved_1000"]["ids"]
    assert client.execute_command("BF.MADD", "bf:students", *ids) == g["replies"]
    links = client.bf_links("bf:students")
    assert [(l["entries"], l["bytes"], l["bits"], l["hashes"], l["size"]) for l in links] == \
        [(l["entries"], l["bytes"], l["bits"], l["hashes"], l["size"]) for l in g["links"]]
    for i in range(len(links)):
        assert np.array_equal(client.bf_link_bits("bf:students", i),
                              golden_arrays[f"default_chain_link{i}"])


def test_madd_one_by_one_equals_batch(pkg, orc):
    """BF.ADD per id (as data_generator.py:58-63 does) == one BF.MADD."""
    rng = np.random.default_rng(3)
    ids = [int(x) for x in rng.integers(10000, 12000, 700)]  # with duplicates
    a = pkg.SketchClient(decode_responses=True)
    b = pkg.SketchClient(decode_responses=True)
    one = [a.execute_command("BF.ADD", "bf", i) for i in ids]
    batch = b.execute_command("BF.MADD", "bf", *ids)
    chain = orc.Chain(100, 0.01)
    want = [chain.add(str(i).encode()) for i in ids]
    assert one == want and batch == want
    assert a.bf_links("bf") == b.bf_links("bf")


def test_madd_nonscaling_full(client, orc):
    client.execute_command("BF.RESERVE", "ns", 0.01, 50, "NONSCALING")
    ids = list(range(5000, 5200))
    got = client.execute_command("BF.MADD", "ns", *ids)
    chain = orc.Chain(50, 0.01, nonscaling=True)
    want = [chain.add(str(i).encode()) for i in ids]
    assert [(-2 if isinstance(r, Exception) else r) for r in got] == want


def test_madd_large_scaling_vs_oracle(client, orc):
    rng = np.random.default_rng(4)
    ids = rng.integers(10**7, 10**8, 120000)
    buf, offs = client_pack(ids)
    client.execute_command("BF.RESERVE", "big", 0.001, 10000, "EXPANSION", 3)
    got = client.bf_madd_packed("big", buf, offs)
    chain = orc.Chain(10000, 0.001, expansion=3)
    want = chain.madd_packed(buf, offs)
    assert np.array_equal(got, want)
    links = client.bf_links("big")
    assert len(links) == chain.nlinks
    for i in range(chain.nlinks):
        assert links[i]["size"] == chain.link_info(i)["size"]
        assert np.array_equal(client.bf_link_bits("big", i), chain.link_bits(i))


# ------------------------------------------------------------------ HLL
def test_pfadd_replies_sequential(client, orc):
    rng = np.random.default_rng(5)
    pipe = client.pipeline()
    calls = []
    for _ in range(400):
        key = f"hll:{int(rng.integers(0, 5))}"
        vals = [int(v) for v in rng.integers(0, 3000, int(rng.integers(0, 4)))]
        pipe.pfadd(key, *vals)
        calls.append((key, vals))
    got = pipe.execute()
    regs, want = {}, []
    for key, vals in calls:
        created = key not in regs
        h = regs.setdefault(key, orc.HLL())
        ch = 0
        for v in vals:
            ch |= h.add(str(v).encode())
        want.append(1 if (created or ch) else 0)
    assert got == want
    for key, h in regs.items():
        assert np.array_equal(client.hll_registers(key), h.regs)
        assert client.pfcount(key) == h.count()


def test_pfadd_docs_examples_on_device(client):
    assert client.pfadd("hll", *"abcdefg") == 1
    assert client.pfcount("hll") == 7
    client.delete("hll")
    client.pfadd("hll", "foo", "bar", "zap")
    client.pfadd("hll", "zap", "zap", "zap")
    client.pfadd("hll", "foo", "bar")
    assert client.pfcount("hll") == 3
    client.pfadd("some-other-hll", 1, 2, 3)
    assert client.pfcount("hll", "some-other-hll") == 6
    client.pfadd("hll1", "foo", "bar", "zap", "a")
    client.pfadd("hll2", "a", "b", "c", "foo")
    assert client.pfmerge("hll3", "hll1", "hll2") is True
    assert client.pfcount("hll3") == 6


def test_pfcount_estimator_exact(client, orc, golden):
    """Device estimator (K2) == Redis hllCount on synthetic register arrays
    from empty to saturated, including H[51] > 0 and H[0] extremes."""
    rng = np.random.default_rng(6)
    arrays = []
    for fill in [0, 1, 3, 30, 300, 3000, 30000, 3 * 10**5, 3 * 10**6, 3 * 10**8, 10**12]:
        n_per = fill / 16384.0
        u = rng.random(16384)
        r = np.ceil(-np.log2(1 - u ** (1.0 / max(n_per, 1e-12)))).clip(0, 51) if fill else np.zeros(16384)
        if fill and fill < 16384:
            r[rng.random(16384) > fill / 16384.0] = 0
        arrays.append(r.astype(np.uint8))
    full = np.full(16384, 51, np.uint8)
    arrays += [full, np.where(rng.random(16384) < 0.5, 51, 1).astype(np.uint8)]
    keys = []
    for i, a in enumerate(arrays):
        client.hll_load_registers(f"k{i}", a)
        keys.append(f"k{i}")
    got = client.pfcount_each(keys)
    want = [orc.hll_count_regs(a) for a in arrays]
    assert got.tolist() == want
    for k, a in zip(keys, arrays):
        h = np.zeros(64, np.uint32)
        client.ctx.call("ske_hll_histogram", client.keys.slot[k.encode()], h.ctypes.data_as(C.c_void_p))
        assert np.array_equal(h, np.bincount(a, minlength=64))


def test_pfcount_groups_and_merge(client, orc):
    rng = np.random.default_rng(7)
    hs = []
    for i in range(12):
        vals = [int(v) for v in rng.integers(0, 10**6, int(rng.integers(0, 20000)))]
        if vals:
            client.pfadd(f"d{i}", *vals)
        else:
            client.pfadd(f"d{i}")
        h = orc.HLL()
        h.add(*[str(v).encode() for v in vals])
        hs.append(h)
    groups = [[f"d{i}" for i in range(j, min(12, j + 4))] for j in range(0, 12, 3)]
    groups.append(["missing", "d0"])
    got = client.pfcount_groups(groups)
    for g, c in zip(groups, got):
        u = orc.HLL()
        for k in g:
            if k != "missing":
                u.merge(hs[int(k[1:])])
        assert int(c) == u.count()
    client.pfmerge("all", *[f"d{i}" for i in range(12)])
    u = orc.HLL()
    for h in hs:
        u.merge(h)
    assert np.array_equal(client.hll_registers("all"), u.regs)
    assert client.hll_dense("all") == u.dense()


# ------------------------------------------------------------------ fused K1
def _oracle_swipes(orc, chain, nkeys, buf, offs, slot):
    regs = np.zeros((nkeys, 16384), np.uint8)
    valid, nvalid, probes = orc.process_swipes(chain, regs, slot, buf, offs)
    return valid, regs, probes


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("pb", [1, 4, 8])
def test_swipes_c2_shape_vs_oracle(engine, orc, variant, pb):
    """Fused BF.EXISTS + PFADD on a C2-shaped stream (7-digit ids, 10 %
    invalid, 50 keys) generated on device: valid flags and all 50 register
    arrays bit-exact."""
    from rtsas_amd import synthetic
    w = synthetic.WORKLOADS["c2"]
    w = synthetic.Workload(**{**w.__dict__, "n_members": 20000, "bf_capacity": 20000})
    engine.set_option("variant", variant)
    engine.set_option("tile", pb)
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    b = engine.swipe_batch(p, 0, 300_000)
    from rtsas_amd.engine import DeviceBuffer
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    buf, offs, slot = b.to_host()
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    valid, regs, probes = _oracle_swipes(orc, chain, w.n_keys, buf, offs, slot)
    assert np.array_equal(out.to_host(np.uint8, b.n), valid)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)
    assert engine.swipes_stats(0, b) == (probes, int(valid.sum()))
    assert engine.variant(0) == variant


@pytest.mark.parametrize("variant", [-1, 0, 2, 3])
def test_swipes_facade_multilink_and_ragged(client, orc, variant):
    """swipes() over a 4-link default chain with ragged ids (0..40 B), keys
    created only when they receive a valid swipe; every K1 variant."""
    client.ctx.call("ske_set_option", b"variant", variant)
    rng = np.random.default_rng(8)
    members = _rand_items(rng, 1000, 40)
    client.execute_command("BF.MADD", "bf", *members)
    chain = orc.Chain(100, 0.01)
    for m in members:
        chain.add(m)
    assert len(client.bf_links("bf")) == chain.nlinks
    items = [members[int(i)] for i in rng.integers(0, 1000, 4000)] + _rand_items(rng, 1000, 40)
    keys = [f"hll:unique:L{int(k)}:2025-03-19" for k in rng.integers(0, 9, len(items))]
    keys += ["hll:never-valid"] * 3
    items += [b"\xff" * 9, b"", b"zz"]
    valid = client.swipes("bf", keys, items)
    want = np.array([bool(chain.exists(x)) for x in items])
    assert np.array_equal(valid, want)
    regs = {}
    for x, k, v in zip(items, keys, want):
        if v:
            regs.setdefault(k, orc.HLL()).add(x)
    for k, h in regs.items():
        assert np.array_equal(client.hll_registers(k), h.regs)
    assert client.exists("hll:never-valid") == (1 if "hll:never-valid" in regs else 0)


def test_swipes_missing_bloom_counts_nothing(client):
    valid = client.swipes("bf:none", "hll:x", [1, 2, 3])
    assert not valid.any()
    assert client.exists("hll:x") == 0


def test_swipes_order_independent_and_idempotent(engine):
    """Registers after a batch do not depend on the order of its swipes, and
    replaying a batch (Pulsar redelivery) changes nothing."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBatch
    w = synthetic.WORKLOADS["c2"]
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(2 * w.n_keys)
    b = engine.swipe_batch(p, 0, 400_000)
    buf, offs, slot = b.to_host()
    engine.swipes(0, b)
    first = engine.registers_all(w.n_keys).copy()
    engine.swipes(0, b)
    assert np.array_equal(engine.registers_all(w.n_keys), first)
    perm = np.random.default_rng(9).permutation(b.n)
    lens = np.diff(offs.astype(np.int64))
    pieces = [buf[offs[i]:offs[i + 1]] for i in perm]
    nbuf = np.concatenate(pieces)
    noffs = np.zeros(b.n + 1, np.uint32)
    noffs[1:] = np.cumsum(lens[perm])
    nslot = slot[perm] + w.n_keys
    b2 = DeviceBatch.from_host(engine.ctx, nbuf, noffs, nslot)
    engine.swipes(0, b2)
    assert np.array_equal(engine.registers_all(2 * w.n_keys)[w.n_keys:], first)


def test_slot_out_of_range_is_an_error(pkg, engine):
    import rtsas_amd
    engine.reserve(0, 0.01, 100)
    engine.hll_reserve(4)
    cap = engine.ctx.lib.ske_hll_capacity(engine.ctx.ptr)
    buf, offs = rtsas_amd.pack_ints([1, 2, 3])
    slot = np.array([0, cap + 5, 1], np.uint32)
    rc = engine.ctx.lib.ske_hll_pfadd(engine.ctx.ptr, slot.ctypes.data_as(C.c_void_p),
                                      buf.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p),
                                      3, None, 0)
    assert rc == -7


def test_sync_call_reports_only_its_own_slot_error(pkg, engine):
    """An enqueue-only K1 with a bad slot is reported by the next ske_sync /
    ske_check_errors, not blamed on a synchronous call that ran clean in
    between (the device word is taken by atomic exchanges, never lost)."""
    import rtsas_amd
    from rtsas_amd._lib import SketchLibError, SKE_ERANGE
    from rtsas_amd.engine import DeviceBatch
    engine.reserve(0, 0.01, 1000)
    buf, offs = rtsas_amd.pack_ints(list(range(100, 200)))
    engine.ctx.call("ske_bf_madd", 0, buf.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p),
                    100, None, 0)
    engine.hll_reserve(4)
    cap = engine.ctx.lib.ske_hll_capacity(engine.ctx.ptr)
    bad = DeviceBatch.from_host(engine.ctx, buf, offs, np.full(100, cap + 3, np.uint32))
    good = DeviceBatch.from_host(engine.ctx, buf, offs, np.zeros(100, np.uint32))
    engine.swipes_async(0, bad)           # leaves the sticky word set
    engine.swipes(0, good)                # synchronous and clean: must not raise
    with pytest.raises(SketchLibError) as ei:
        engine.check_errors()             # the earlier async error surfaces here
    assert ei.value.code == SKE_ERANGE
    engine.check_errors()                 # and only once
    with pytest.raises(SketchLibError):
        engine.swipes(0, bad)             # a synchronous call's own error
    engine.sync()
    bad.free()
    good.free()


def test_generator_matches_numpy_restatement(engine):
    from gen_ref import Gen
    from rtsas_amd import synthetic
    for name, n in [("c2", 50_000), ("c4", 50_000), ("c3", 50_000)]:
        w = synthetic.WORKLOADS[name]
        p = engine.gen_params(w, seed=12345)
        b = engine.swipe_batch(p, 1_000_000, n)
        buf, offs, slot = b.to_host()
        g = Gen(p)
        ids = g.swipe_ids(1_000_000, n)
        wb, wo = g.encode(ids)
        assert np.array_equal(offs, wo)
        assert np.array_equal(buf, wb)
        assert np.array_equal(slot, g.swipe_slots(1_000_000, n, synthetic.key_cdf(w)))
        m = engine.members_batch(p, 500, 1000).to_host()
        mb, mo = g.encode(g.member(np.arange(500, 1500)))
        assert np.array_equal(m[0], mb)
        inv = ~g.is_member(ids)
        assert abs(inv.mean() - w.invalid_frac) < 0.02


def test_empty_and_single(client):
    assert client.execute_command("BF.MADD", "bf", 5) == [1]
    assert client.swipes("bf", "hll:a", []).size == 0
    assert client.swipes("bf", "hll:a", [5]).tolist() == [True]
    assert client.pfcount("hll:a") == 1


def test_hll_get_set_interop(client, orc):
    """GET of an HLL key gives a Redis HYLL string the oracle decodes to the
    same registers; SET of that string into another key reproduces them."""
    vals = list(range(50000, 52000))
    client.pfadd("hll:a", *vals)
    s = client.execute_command("GET", "hll:a")
    regs = orc.hll_decode_string(s)
    h = orc.HLL()
    h.add(*[str(v).encode() for v in vals])
    assert np.array_equal(regs, h.regs)
    assert client.execute_command("SET", "hll:b", s) == "OK"
    assert np.array_equal(client.hll_registers("hll:b"), h.regs)
    assert client.pfcount("hll:b") == h.count()


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_swipes_fixed_width_equals_offsets(engine, orc, variant):
    """ske_swipes_fixed (ids at bytes + i*width, no offsets) == ske_swipes on
    the same batch == the oracle, registers and flags."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c4"]
    engine.set_option("variant", variant)
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(2 * w.n_keys)
    b = engine.swipe_batch(p, 0, 250_000)
    buf, offs, slot = b.to_host()
    o1, o2 = DeviceBuffer(engine.ctx, b.n), DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, o1)
    b.slot.from_host(slot + w.n_keys)           # second copy of the keys
    engine.swipes_fixed(0, b, o2)
    regs = engine.registers_all(2 * w.n_keys)
    assert np.array_equal(o1.to_host(np.uint8, b.n), o2.to_host(np.uint8, b.n))
    assert np.array_equal(regs[:w.n_keys], regs[w.n_keys:])
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    valid, oregs, _ = _oracle_swipes(orc, chain, w.n_keys, buf, offs, slot)
    assert np.array_equal(o2.to_host(np.uint8, b.n), valid)
    assert np.array_equal(regs[w.n_keys:], oregs)


@pytest.mark.parametrize("variant", [-1, 2])
def test_swipes_c3_filter_vs_oracle(engine, orc, variant):
    """K1 at C3's real filter size (RESERVE 0.001 / 1e7: 19.8 MB, 158M bits,
    k = 11) on a 1.5M-swipe slice of the C3 stream (Zipf keys), bit-exact vs
    the oracle: the default partitioned K1 (302 LDS slices of 64 KiB) and the
    XCD-partitioned one (L2 slices of ~2.5 MB); and equal to the global-Bloom
    variant on the same batch."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c3"]
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    assert engine.variant(0) == 3
    engine.set_option("variant", variant)
    assert engine.variant(0) == (3 if variant == -1 else variant)
    keys = 2000  # the stream's first keys only: keep the oracle's slab small
    w_small = synthetic.Workload(**{**w.__dict__, "n_keys": keys, "zipf_lectures": 20,
                                    "zipf_days": 100})
    ps = engine.gen_params(w_small)
    engine.hll_reserve(2 * keys)
    b = engine.swipe_batch(ps, 5_000_000, 1_500_000)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    buf, offs, slot = b.to_host()
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    chain.madd_packed(mb[0], mb[1])
    assert np.array_equal(engine.bloom_bits(0, 0, chain.link_info(0)["bytes"]), chain.link_bits(0))
    valid, regs, _ = _oracle_swipes(orc, chain, keys, buf, offs, slot)
    assert np.array_equal(out.to_host(np.uint8, b.n), valid)
    assert np.array_equal(engine.registers_all(keys), regs)
    # global variant on the same batch into the second half of the slab
    engine.set_option("variant", 0)
    b.slot.from_host(slot + keys)
    out2 = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out2)
    assert np.array_equal(out2.to_host(np.uint8, b.n), valid)
    assert np.array_equal(engine.registers_all(2 * keys)[keys:], regs)


def test_graph_replay_equals_eager(engine):
    """K1 recorded into a HIP graph (ske_capture_begin/end) and replayed over
    four resident batches gives the same registers and answers as the same
    launches made one by one."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c2"]
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(2 * w.n_keys)
    bs = [engine.swipe_batch(p, j * 200_000, 200_000) for j in range(4)]
    outs = [DeviceBuffer(engine.ctx, b.n) for b in bs]
    for b, o in zip(bs, outs):
        engine.swipes_async(0, b, o)
    engine.sync()
    eager = engine.registers_all(w.n_keys).copy()
    answers = [o.to_host(np.uint8, b.n) for b, o in zip(bs, outs)]
    for b in bs:
        b.slot.from_host(b.slot.to_host(np.uint32, b.n) + w.n_keys)
    g = engine.capture(lambda: [engine.swipes_async(0, b, o) for b, o in zip(bs, outs)])
    for o in outs:
        o.from_host(np.full(o.nbytes, 7, np.uint8))
    g.launch()
    engine.sync()
    g.free()
    assert np.array_equal(engine.registers_all(2 * w.n_keys)[w.n_keys:], eager)
    for a, b, o in zip(answers, bs, outs):
        assert np.array_equal(o.to_host(np.uint8, b.n), a)


def test_capture_survives_cyclic_garbage(engine):
    """An unreachable Context in a reference cycle (a test's or a caller's
    engine) must not be finalised inside a stream capture: ske_close's
    hipStreamSynchronize / hipFree there invalidate a thread-local capture
    (round 6: a full-size test's graph recording failed right after a test
    whose engines were left to the cyclic collector).  With the collector
    forced to run on every allocation, the recording still succeeds and the
    replay equals the eager run."""
    import gc
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer, SketchEngine
    w = synthetic.WORKLOADS["c2"]
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    bs = [engine.swipe_batch(p, j * 100_000, 100_000) for j in range(2)]
    outs = [DeviceBuffer(engine.ctx, b.n) for b in bs]
    for b, o in zip(bs, outs):
        engine.swipes_async(0, b, o)
    engine.sync()
    answers = [o.to_host(np.uint8, b.n) for b, o in zip(bs, outs)]
    regs = engine.registers_all(w.n_keys).copy()
    gc.collect()
    old = gc.get_threshold()
    try:
        for _ in range(3):  # unreachable engines in cycles, left to the collector
            other = SketchEngine(0)
            other.hll_reserve(8)
            cyc = [other]
            cyc.append(cyc)
            del other, cyc
        gc.set_threshold(1)  # a collection at (almost) every allocation
        g = engine.capture(lambda: [engine.swipes_async(0, b, o) for b, o in zip(bs, outs)])
    finally:
        gc.set_threshold(*old)
    gc.collect()
    g.launch()
    engine.sync()
    g.free()
    assert np.array_equal(engine.registers_all(w.n_keys), regs)  # the replay raises nothing new
    for a, b, o in zip(answers, bs, outs):
        assert np.array_equal(o.to_host(np.uint8, b.n), a)


@pytest.mark.parametrize("variant", [-1, 2, 3])
def test_two_streams_equal_one_stream(engine, variant):
    """Launches alternating over two HIP streams (overlapping K1 kernels; the
    XCD-partitioned variant serialises on its scratch) leave the same
    registers and answers as the same launches on one stream."""
    import torch
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c2"]
    engine.set_option("variant", variant)
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(2 * w.n_keys)
    bs = [engine.swipe_batch(p, j * 150_000, 150_000) for j in range(6)]
    outs = [DeviceBuffer(engine.ctx, b.n) for b in bs]
    for b, o in zip(bs, outs):
        engine.swipes_async(0, b, o)
    engine.sync()
    one = engine.registers_all(w.n_keys).copy()
    answers = [o.to_host(np.uint8, b.n) for b, o in zip(bs, outs)]
    for b in bs:
        b.slot.from_host(b.slot.to_host(np.uint32, b.n) + w.n_keys)
    st = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for j, (b, o) in enumerate(zip(bs, outs)):
        engine.set_stream(st[j % 2].cuda_stream)
        engine.swipes_async(0, b, o)
    torch.cuda.synchronize()
    engine.set_stream(None)
    assert np.array_equal(engine.registers_all(2 * w.n_keys)[w.n_keys:], one)
    for a, b, o in zip(answers, bs, outs):
        assert np.array_equal(o.to_host(np.uint8, b.n), a)


@pytest.mark.parametrize("shape", ["default-chain", "c3-filter"])
def test_bf_scandump_loadchunk_round_trip(client, orc, shape):
    """BF.SCANDUMP of a chain (header chunk, then bit-array chunks of at most
    MAX_SCANDUMP_SIZE bytes, then (0, b'')) replayed by BF.LOADCHUNK into
    another key gives the same links, bit arrays, BF.INFO and answers."""
    rng = np.random.default_rng(11)
    if shape == "default-chain":
        ids = [int(x) for x in rng.choice(np.arange(10000, 99999), 1000, replace=False)]
        client.execute_command("BF.MADD", "src", *ids)   # auto-created, grows to 4 links
    else:
        client.execute_command("BF.RESERVE", "src", 0.001, 10_000_000)  # 19.8 MB: 2 chunks
        ids = [int(x) for x in rng.integers(10**7, 10**8, 200_000)]
        client.bf_madd_packed("src", *client_pack(ids))
    chunks, it = [], 0
    while True:
        it, data = client.execute_command("BF.SCANDUMP", "src", it)
        if it == 0:
            assert data == b""
            break
        chunks.append((it, data))
    assert all(len(d) <= client.MAX_SCANDUMP_SIZE for _, d in chunks[1:])
    for it, data in chunks:
        assert client.execute_command("BF.LOADCHUNK", "dst", it, data) == "OK"
    assert client.bf_links("dst") == client.bf_links("src")
    assert client.bf_info("dst") == client.bf_info("src")
    for i in range(len(client.bf_links("src"))):
        assert np.array_equal(client.bf_link_bits("dst", i), client.bf_link_bits("src", i))
    probe = ids[:5000] + [int(x) for x in rng.integers(10**7, 10**8, 5000)]
    assert client.execute_command("BF.MEXISTS", "dst", *probe) == \
        client.execute_command("BF.MEXISTS", "src", *probe)
    with pytest.raises(Exception, match="item exists"):
        client.execute_command("BF.LOADCHUNK", "dst", 1, chunks[0][1])


@pytest.mark.parametrize("shape", ["default-chain", "c3-filter"])
def test_bf_loadchunk_of_oracle_dump(client, orc, shape):
    """BF.LOADCHUNK of a dump the ORACLE produced (oracle/sketch_oracle.c's
    restatement of RedisBloom SBChain_GetEncodedHeader / GetEncodedChunk, an
    encoder independent of formats.py): the reference's default 4-link chain
    (1000 ids BF.ADDed to an auto-created key, data_generator.py:57-63) and
    the C3 filter.  The device chain must then have the oracle's BF.INFO,
    every link's bits, and its MEXISTS answers; and the device's own
    BF.SCANDUMP must reproduce the oracle's chunks byte for byte.  Parity
    unpinned vs a live RedisBloom (layout [recall])."""
    rng = np.random.default_rng(23)
    if shape == "default-chain":
        ch = orc.Chain(100, 0.01)
        ids = [int(x) for x in rng.choice(np.arange(10000, 100000), 1000, replace=False)]
        for i in ids:
            ch.add(str(i).encode())
        assert ch.nlinks == 4
        probe = ids + [int(x) for x in rng.integers(100000, 999999, 3000)]
    else:
        ch = orc.Chain(10_000_000, 0.001)
        ids = rng.integers(10**7, 10**8, 300_000)
        ch.madd_packed(*client_pack([int(x) for x in ids]))
        probe = [int(x) for x in ids[:50_000]] + [int(x) for x in rng.integers(10**7, 10**8, 50_000)]
    dump = ch.scandump_all(max_chunk=4096 if shape == "default-chain" else orc.MAX_SCANDUMP_SIZE)
    for it, data in dump:
        assert client.execute_command("BF.LOADCHUNK", "ld", it, data) == "OK"
    info = client.bf_info("ld")
    assert info["Number of filters"] == ch.nlinks
    assert info["Number of items inserted"] == ch.size
    links = client.bf_links("ld")
    for i in range(ch.nlinks):
        o = ch.link_info(i)
        assert {k: links[i][k] for k in ("entries", "bytes", "bits", "hashes", "size")} == \
            {k: o[k] for k in ("entries", "bytes", "bits", "hashes", "size")}, i
        assert links[i]["error"] == o["error"]
        assert np.array_equal(client.bf_link_bits("ld", i), ch.link_bits(i)), f"link {i} bits"
    pb, po = client_pack(probe)
    want, _ = ch.mexists_packed(pb, po)
    assert client.execute_command("BF.MEXISTS", "ld", *probe) == want.astype(int).tolist()
    got, it = [], 0
    while True:
        it, data = client.execute_command("BF.SCANDUMP", "ld", it)
        if it == 0:
            break
        got.append((it, data))
    assert got == ch.scandump_all()


def test_pfmerge_many_sources_two_level(client):
    """PFMERGE of 3000 keys (the two-level parallel merge used past 256
    sources) == the register-wise max, dst's own registers included; and
    PFCOUNT of every key with a null slot list (keys 0..n-1)."""
    rng = np.random.default_rng(12)
    arrays = rng.integers(0, 20, (3000, 16384)).astype(np.uint8)
    arrays[rng.random(arrays.shape) < 0.9] = 0
    arrays[17, 5] = 51
    for i, a in enumerate(arrays):
        client.hll_load_registers(f"day{i}", a)
    dst_own = rng.integers(0, 3, 16384).astype(np.uint8)
    dst_own[9] = 50
    client.hll_load_registers("campus", dst_own)
    assert client.pfmerge("campus", *[f"day{i}" for i in range(3000)]) is True
    want = np.maximum(arrays.max(axis=0), dst_own)
    assert np.array_equal(client.hll_registers("campus"), want)
    import ctypes as C
    n = client.ctx.lib.ske_hll_capacity(client.ctx.ptr)
    out = np.zeros(n, np.uint64)
    client.ctx.call("ske_hll_pfcount_each", None, n, out.ctypes.data_as(C.c_void_p), 0)
    slots = [client.keys.slot[f"day{i}".encode()] for i in range(0, 3000, 250)]
    assert [int(out[s]) for s in slots] == client.pfcount_each([f"day{i}" for i in range(0, 3000, 250)]).tolist()


@pytest.mark.parametrize("variant", [-1, 3])
def test_property_swipes_vs_oracle(pkg, orc, variant):
    """Hypothesis: fused swipes on random byte ids (0..64 B), random key skews
    and batch sizes from 0 to a few thousand == the oracle's sequential
    BF.EXISTS + PFADD, answers and registers; through the variant the library
    picks (the LDS K1 for this filter) and through the partitioned K1 forced
    (variant 3: ragged tiles, empty and long ids through its generic hash)."""
    from hypothesis import HealthCheck, given, settings, strategies as st
    client = pkg.SketchClient(decode_responses=True)
    if variant >= 0:
        client.ctx.call("ske_set_option", b"variant", variant)
    members = [bytes([i % 256, i // 256, 7]) * (1 + i % 5) for i in range(3000)]
    client.execute_command("BF.RESERVE", "bf", 0.01, 5000)
    client.execute_command("BF.MADD", "bf", *members)
    chain = orc.Chain(5000, 0.01)
    for m in members:
        chain.add(m)
    counter = [0]

    @settings(max_examples=25, deadline=None, suppress_health_check=list(HealthCheck))
    @given(st.lists(st.one_of(st.binary(min_size=0, max_size=64), st.sampled_from(members)),
                    min_size=0, max_size=3000),
           st.integers(1, 40), st.floats(0.0, 3.0))
    def run(items, nkeys, skew):
        counter[0] += 1
        rng = np.random.default_rng(counter[0])
        w = 1.0 / np.arange(1, nkeys + 1) ** skew
        kid = rng.choice(nkeys, size=len(items), p=w / w.sum())
        keys = [f"h{counter[0]}:{int(k)}" for k in kid]
        valid = client.swipes("bf", keys, items)
        regs = {}
        for x, k in zip(items, keys):
            if chain.exists(x):
                regs.setdefault(k, orc.HLL()).add(x)
        assert valid.tolist() == [bool(chain.exists(x)) for x in items]
        for k, h in regs.items():
            assert np.array_equal(client.hll_registers(k), h.regs)

    run()


def test_pfcount_each_many_keys_vs_oracle(client, orc):
    """PFCOUNT of every key over more keys than the wave-per-key kernel has
    waves (each wave bins several keys into running-total columns), in slab
    order (null slot list) and in a shuffled key order: every count ==
    Redis's hllCount on the same registers."""
    rng = np.random.default_rng(21)
    n = 5000
    fill = rng.integers(0, 6, n)
    arrays = np.zeros((n, 16384), np.uint8)
    for i in range(n):
        dens = [0.0, 0.01, 0.1, 0.5, 0.9, 1.0][fill[i]]
        vals = rng.geometric(0.5, 16384).clip(1, 51)
        arrays[i] = np.where(rng.random(16384) < dens, vals, 0)
    arrays[7] = 51
    arrays[8] = 0
    names = [f"k{i}" for i in range(n)]
    for k, a in zip(names, arrays):
        client.hll_load_registers(k, a)
    want = np.array([orc.hll_count_regs(a) for a in arrays], np.uint64)
    order = rng.permutation(n)
    got = client.pfcount_each([names[i] for i in order])
    assert np.array_equal(got, want[order])
    slots = np.array([client.keys.slot[k.encode()] for k in names])
    cap = client.ctx.lib.ske_hll_capacity(client.ctx.ptr)
    out = np.zeros(cap, np.uint64)
    client.ctx.call("ske_hll_pfcount_each", None, cap, out.ctypes.data_as(C.c_void_p), 0)
    assert np.array_equal(out[slots], want)


def test_host_staged_swipes_reject_decreasing_offsets(engine, pkg, orc):
    """ske_swipes with host buffers (SKE_MEM_HOST) checks the offsets while the
    copies run: decreasing offsets return SKE_EINVAL before any kernel reads
    them (registers untouched); a valid call right after answers == the oracle."""
    from rtsas_amd._lib import SKE_EINVAL, SKE_MEM_HOST
    rng = np.random.default_rng(11)
    engine.reserve(0, 0.01, 10_000)
    members = [b"%d" % v for v in rng.choice(np.arange(10**6, 10**7), 5000, replace=False)]
    buf = np.frombuffer(b"".join(members), np.uint8).copy()
    offs = np.concatenate([[0], np.cumsum([len(m) for m in members])]).astype(np.uint32)
    engine.ctx.call("ske_bf_madd", 0, C.c_void_p(buf.ctypes.data), C.c_void_p(offs.ctypes.data),
                    len(members), None, SKE_MEM_HOST)
    engine.hll_reserve(8)
    n = 4000
    items = members[:2000] + [b"%d" % v for v in rng.integers(10**7, 10**8, 2000)]
    ib = np.frombuffer(b"".join(items), np.uint8).copy()
    io = np.concatenate([[0], np.cumsum([len(x) for x in items])]).astype(np.uint32)
    slot = rng.integers(0, 8, n).astype(np.uint32)
    out = np.zeros(n, np.uint8)
    bad = io.copy()
    bad[1000], bad[1001] = bad[1001], bad[1000]
    ptr = lambda a: C.c_void_p(a.ctypes.data)
    with pytest.raises(pkg.SketchLibError) as ei:
        engine.ctx.call("ske_swipes", 0, ptr(slot), ptr(ib), ptr(bad), n, ptr(out), SKE_MEM_HOST)
    assert ei.value.code == SKE_EINVAL
    assert not engine.registers_all(8).any()
    engine.ctx.call("ske_swipes", 0, ptr(slot), ptr(ib), ptr(io), n, ptr(out), SKE_MEM_HOST)
    chain = orc.Chain(10_000, 0.01)
    chain.madd_packed(buf, offs)
    regs = np.zeros((8, 16384), np.uint8)
    want, _, _ = orc.process_swipes(chain, regs, slot, ib, io)
    assert np.array_equal(out, want)
    assert np.array_equal(engine.registers_all(8), regs)


@pytest.mark.parametrize("defect", [None, "mid-slice", "slice-boundary", "chunk-boundary"])
def test_host_staged_large_offsets_checked_on_the_pinned_copy(engine, pkg, orc, defect):
    """Pageable offsets above 8 MB go through the copy threads and the pinned
    double buffer (sketch_host.cpp): the monotone check runs on the copy the
    DMA moves.  A clean 12M-swipe batch (48 MB of offsets: two 32 MB chunks, 8
    thread slices each) answers == the device path; one decrease inside a
    thread's slice, exactly at a slice boundary, or at the chunk boundary is
    refused (SKE_EINVAL) with the registers untouched."""
    from rtsas_amd._lib import SKE_EINVAL, SKE_MEM_HOST
    from rtsas_amd.engine import DeviceBatch, DeviceBuffer
    rng = np.random.default_rng(3)
    engine.reserve(0, 0.01, 100_000)
    members = rng.choice(np.arange(10**6, 10**7), 50_000, replace=False)
    mb, mo = pkg.pack_ints(members)
    engine.ctx.call("ske_bf_madd", 0, C.c_void_p(mb.ctypes.data), C.c_void_p(mo.ctypes.data),
                    members.size, None, SKE_MEM_HOST)
    engine.hll_reserve(16)
    n = 12_000_000
    ids = np.where(rng.random(n) < 0.9, rng.choice(members, n), rng.integers(10**6, 10**7, n))
    buf, offs = pkg.pack_ints(ids)
    slot = rng.integers(0, 16, n).astype(np.uint32)
    out = np.zeros(n, np.uint8)
    ptr = lambda a: C.c_void_p(a.ctypes.data)
    if defect is not None:
        bad = offs.copy()
        # 32 MB chunks of u32 = 8M elements; 8 slices of 4 MB = 1M elements
        k = {"mid-slice": 1_234_567, "slice-boundary": 3 << 20, "chunk-boundary": 8 << 20}[defect]
        bad[k] = bad[k - 1] - 1
        with pytest.raises(pkg.SketchLibError) as ei:
            engine.ctx.call("ske_swipes", 0, ptr(slot), ptr(buf), ptr(bad), n, ptr(out), SKE_MEM_HOST)
        assert ei.value.code == SKE_EINVAL
        assert not engine.registers_all(16).any()
        return
    engine.ctx.call("ske_swipes", 0, ptr(slot), ptr(buf), ptr(offs), n, ptr(out), SKE_MEM_HOST)
    regs_host = engine.registers_all(16)
    from rtsas_amd.engine import SketchEngine
    e2 = SketchEngine(0)
    e2.reserve(0, 0.01, 100_000)
    e2.ctx.call("ske_bf_madd", 0, C.c_void_p(mb.ctypes.data), C.c_void_p(mo.ctypes.data),
                members.size, None, SKE_MEM_HOST)
    e2.hll_reserve(16)
    b = DeviceBatch.from_host(e2.ctx, buf, offs, slot)
    dout = DeviceBuffer(e2.ctx, n)
    e2.swipes(0, b, dout)
    assert np.array_equal(out, dout.to_host(np.uint8, n))
    assert np.array_equal(regs_host, e2.registers_all(16))


def test_product_options_only(engine):
    """The shipped library takes only the six tuning options; the diagnostic
    and measured-slower knobs of earlier rounds (ablate, hll_mode,
    part_overlap, ...) are gone and refused: no option can
    make an answer or a register wrong."""
    from rtsas_amd._lib import SKE_EINVAL
    lib, ptr = engine.ctx.lib, engine.ctx.ptr
    for name in [b"ablate", b"hll_mode", b"part_overlap", b"part_ccus", b"pa_tile", b"pa_precheck",
                 b"pa_grid", b"pa_threads", b"pb_pairs", b"k1_legacy", b"xr_region_u", b"xr_finish_u"]:
        assert lib.ske_set_option(ptr, name, 1) == SKE_EINVAL, name
    for name, val in [(b"variant", -1), (b"tile", 2), (b"k1_grid", 0), (b"k1_persistent", 1),
                      (b"part_sub", 0), (b"pass_timing", 0)]:
        assert lib.ske_set_option(ptr, name, val) == 0, name
    assert lib.ske_set_option(ptr, b"tile", 3) == SKE_EINVAL
