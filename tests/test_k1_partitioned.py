"""The partitioned K1 (sketch_part.hip) beyond the shared variant tests, the
error channel of the enqueue-only calls, and graph / scratch safety.

- multi-link chains through the partitioned kernel (links of different k,
  slices numbered across links), ragged ids of 0..40 bytes;
- ske_swipes_many_async with an out-of-range HLL slot, enqueued directly and
  recorded into a graph: the sticky device error word surfaces as SKE_ERANGE
  at ske_check_errors / ske_sync (the swipe's BF.EXISTS answer is still
  written; its PFADD is dropped), and the next call starts clean;
- a graph replay followed at once by a direct launch on a second stream:
  both use the context scratch, the direct launch waits for the replay
  (ADVICE r1), answers and registers == the oracle.

Every check is bit-exact against the oracle (oracle/sketch_oracle.c, the
restatement of RedisBloom SBChain_Check + Redis hllAdd that
attendance_processor.py:109-113 / :127-129 reach).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rand_items(rng, n, maxlen, minlen=0):
    lens = rng.integers(minlen, maxlen + 1, n)
    return [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]


def _pack(items):
    offs = np.zeros(len(items) + 1, np.uint32)
    offs[1:] = np.cumsum([len(x) for x in items])
    buf = np.frombuffer(b"".join(items) + b"\0" * 16, np.uint8).copy()
    return buf, offs


def test_partitioned_two_link_chain_ragged(engine, orc):
    """RESERVE 0.01 / 20000 grown to two links (k = 8, 9: 17 probes per swipe,
    tiles of 1024 swipes), ragged ids; the partitioned kernel forced (the
    general instantiation: k_part_a<22>, single-slice k_part_b<1>, fail
    bytes, k_part_c)."""
    from rtsas_amd.engine import DeviceBatch, DeviceBuffer
    rng = np.random.default_rng(21)
    members = _rand_items(rng, 30000, 40, 1)
    engine.reserve(0, 0.01, 20000)
    mb, mo = _pack(members)
    dm = DeviceBatch.from_host(engine.ctx, mb, mo, np.zeros(len(members), np.uint32))
    import ctypes as C
    engine.ctx.call("ske_bf_madd", 0, C.c_void_p(dm.bytes.ptr), C.c_void_p(dm.offs.ptr),
                    len(members), None, 1)
    chain = orc.Chain(20000, 0.01)
    chain.madd_packed(mb, mo)
    assert chain.nlinks == 2
    engine.set_option("variant", 3)
    assert engine.variant(0) == 3
    items = [members[int(i)] for i in rng.integers(0, len(members), 60000)]
    items += _rand_items(rng, 20000, 40)
    items += [b"", b"x"]
    keys = rng.integers(0, 37, len(items)).astype(np.uint32)
    buf, offs = _pack(items)
    engine.hll_reserve(37)
    b = DeviceBatch.from_host(engine.ctx, buf, offs, keys)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    regs = np.zeros((37, 16384), np.uint8)
    valid, _, _ = orc.process_swipes(chain, regs, keys, buf, offs)
    assert np.array_equal(out.to_host(np.uint8, b.n), valid)
    assert np.array_equal(engine.registers_all(37), regs)


def test_c3_geometry_ragged_long_ids(engine, orc):
    """The one-link k = 11 chain of C3's RESERVE 0.001 / 1e7 (the fail-list
    path: k_part_a3, k_part_b<2, 4, true>, k_part_c_fl) on ids of 0..40
    bytes: empty ids and ids longer than 8 bytes take pass A's generic
    MurmurHash64A; a ragged last tile; answers and registers == the oracle."""
    from rtsas_amd.engine import DeviceBatch, DeviceBuffer
    import ctypes as C
    rng = np.random.default_rng(77)
    members = _rand_items(rng, 40000, 40, 1)
    engine.reserve(0, 0.001, 10_000_000)
    mb, mo = _pack(members)
    dm = DeviceBatch.from_host(engine.ctx, mb, mo, np.zeros(len(members), np.uint32))
    engine.ctx.call("ske_bf_madd", 0, C.c_void_p(dm.bytes.ptr), C.c_void_p(dm.offs.ptr), len(members), None, 1)
    chain = orc.Chain(10_000_000, 0.001)
    chain.madd_packed(mb, mo)
    assert chain.nlinks == 1 and chain.link_info(0)["hashes"] == 11
    assert engine.variant(0) == 3
    items = [members[int(i)] for i in rng.integers(0, len(members), 90000)]
    items += _rand_items(rng, 30000, 40) + [b""] * 50 + [b"12345678", b"123456789"]
    order = rng.permutation(len(items))
    items = [items[int(i)] for i in order]
    keys = rng.integers(0, 37, len(items)).astype(np.uint32)
    buf, offs = _pack(items)
    engine.hll_reserve(37)
    b = DeviceBatch.from_host(engine.ctx, buf, offs, keys)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    regs = np.zeros((37, 16384), np.uint8)
    valid, _, _ = orc.process_swipes(chain, regs, keys, buf, offs)
    assert np.array_equal(out.to_host(np.uint8, b.n), valid)
    assert np.array_equal(engine.registers_all(37), regs)
    assert valid.sum() > 80000


def _c3_small(engine, n_members=200_000):
    from rtsas_amd import synthetic
    w = synthetic.WORKLOADS["c3"]
    w = synthetic.Workload(**{**w.__dict__, "n_members": n_members, "n_keys": 64,
                              "zipf_lectures": 0, "zipf_days": 0})
    engine.reserve(0, w.bf_error, w.bf_capacity)   # the 19.8 MB C3 geometry
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    assert engine.variant(0) == 3
    return w, p


@pytest.mark.parametrize("mode", ["direct", "graph"])
def test_many_async_out_of_range_slot_surfaces(engine, orc, mode):
    import torch
    from rtsas_amd._lib import SketchLibError, SKE_ERANGE
    from rtsas_amd.engine import DeviceBuffer
    w, p = _c3_small(engine)
    cap = engine.ctx.lib.ske_hll_capacity(engine.ctx.ptr)
    bs = [engine.swipe_batch(p, j * 300_000, 300_000) for j in range(3)]
    good = [b.slot.to_host(np.uint32, b.n) for b in bs]
    bad = good[1].copy()
    bad[12345] = cap + 7          # one swipe names a slot past the slab
    bs[1].slot.from_host(bad)
    outs = [DeviceBuffer(engine.ctx, b.n) for b in bs]
    main = torch.cuda.Stream()
    engine.set_stream(main.cuda_stream)
    try:
        engine.swipes_many_async(0, [], branches=2)
        if mode == "direct":
            engine.swipes_many_async(0, bs, outs, branches=2)
        else:
            engine.swipes_many_async(0, bs[:1], outs[:1], branches=1)  # sizes the scratch
            torch.cuda.synchronize()
            g = engine.capture(lambda: engine.swipes_many_async(0, bs, outs, branches=2))
            g.launch()
        with pytest.raises(SketchLibError) as ei:
            engine.check_errors()
        assert ei.value.code == SKE_ERANGE
        engine.check_errors()     # cleared: the next check is clean
        if mode == "graph":
            g.free()
    finally:
        engine.set_stream(None)
    # answers are still BF.EXISTS for every swipe; the bad swipe's PFADD is
    # dropped (the oracle sends it to a spare row that is not compared)
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    regs = np.zeros((w.n_keys + 1, 16384), np.uint8)
    for j, b in enumerate(bs):
        buf, offs, _ = b.to_host()
        sl = good[j].copy()
        if j == 1:
            sl[12345] = w.n_keys
        v, _, _ = orc.process_swipes(chain, regs, sl, buf, offs)
        assert np.array_equal(outs[j].to_host(np.uint8, b.n), v)
    assert np.array_equal(engine.registers_all(w.n_keys), regs[:w.n_keys])


def test_graph_replay_then_direct_launch_other_stream(engine, orc):
    """A replayed graph holding the partitioned K1 and a direct K1 launch on
    a second stream right behind it share the scratch: the direct launch
    waits for the replay."""
    import torch
    from rtsas_amd.engine import DeviceBuffer
    w, p = _c3_small(engine)
    bs = [engine.swipe_batch(p, j * 1_200_000, 1_200_000) for j in range(3)]  # > 512 tiles each
    outs = [DeviceBuffer(engine.ctx, b.n) for b in bs]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    engine.set_stream(s1.cuda_stream)
    try:
        engine.swipes_async(0, bs[0], outs[0])
        torch.cuda.synchronize()
        g = engine.capture(lambda: [engine.swipes_async(0, b, o) for b, o in zip(bs[:2], outs[:2])])
        g.launch()
        engine.set_stream(s2.cuda_stream)
        engine.swipes_async(0, bs[2], outs[2])
        torch.cuda.synchronize()
        g.free()
    finally:
        engine.set_stream(None)
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    for b, o in zip(bs, outs):
        buf, offs, slot = b.to_host()
        v, _, _ = orc.process_swipes(chain, regs, slot.astype(np.uint32), buf, offs)
        assert np.array_equal(o.to_host(np.uint8, b.n), v)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


@pytest.mark.parametrize("invalid", [0.1, 0.5, 1.0])
@pytest.mark.parametrize("error", [0.001, 0.0001])
def test_fail_lists_and_overflow_vs_oracle(engine, orc, invalid, error):
    """error 0.001 (C3's filter, one link of k = 11): pass B -> C through fail
    lists; at 100 % invalid every (slice pair, tile) list overflows into the
    fail bytes many times over, at 10 % a few do.  error 0.0001 (one link of
    k = 15, 394 slices): the general instantiation on slice pairs (k_part_a<22>,
    k_part_b<2>, fail bytes, k_part_c).  A ragged last tile; answers and
    registers == the oracle."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c3"]
    w = synthetic.Workload(**{**w.__dict__, "n_members": 300_000, "n_keys": 97, "zipf_lectures": 0,
                              "zipf_days": 0, "invalid_frac": invalid, "bf_error": error})
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w, seed=4242)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    assert engine.variant(0) == 3
    b = engine.swipe_batch(p, 7, 700_000 + 333)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    buf, offs, slot = b.to_host()
    v, nvalid, _ = orc.process_swipes(chain, regs, slot.astype(np.uint32), buf, offs)
    assert np.array_equal(out.to_host(np.uint8, b.n), v)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)
    if invalid == 1.0:
        assert nvalid < b.n // 500   # only Bloom false positives remain


@pytest.mark.parametrize("invalid", [0.1, 1.0])
@pytest.mark.parametrize("capacity", [10_000_000, 20_000_000, 40_000_000])
def test_pass_a_counter_layouts_vs_oracle(engine, orc, invalid, capacity):
    """The fail-list pass A's two counter tables: 1024 counters (two per
    thread) for chains under 512 slice pairs (C3's 1e7 filter: 303 slices,
    2e7: 604) and 2048 for longer ones (4e7: over 1100 slices); a ragged last
    tile; answers and registers == the oracle."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c3"]
    w = synthetic.Workload(**{**w.__dict__, "n_members": 300_000, "n_keys": 97, "zipf_lectures": 0,
                              "zipf_days": 0, "invalid_frac": invalid, "bf_capacity": capacity})
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w, seed=4243)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    assert engine.variant(0) == 3
    b = engine.swipe_batch(p, 11, 900_000 + 517)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    buf, offs, slot = b.to_host()
    v, _, _ = orc.process_swipes(chain, regs, slot.astype(np.uint32), buf, offs)
    assert np.array_equal(out.to_host(np.uint8, b.n), v)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


def test_hll_reserve_refused_while_graph_alive(engine):
    from rtsas_amd._lib import SketchLibError, SKE_EBUSY
    from rtsas_amd.engine import DeviceBuffer
    w, p = _c3_small(engine, n_members=10_000)
    b = engine.swipe_batch(p, 0, 100_000)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    g = engine.capture(lambda: engine.swipes_async(0, b, out))
    cap = engine.ctx.lib.ske_hll_capacity(engine.ctx.ptr)
    with pytest.raises(SketchLibError) as ei:
        engine.hll_reserve(cap + 100)
    assert ei.value.code == SKE_EBUSY
    g.launch()
    engine.sync()
    g.free()
    engine.hll_reserve(cap + 100)  # no graph holds the slab any more


def test_partitioned_hot_register_and_many_keys(engine, orc):
    """Adversarial PFADD shapes for pass C's CAS: 2M swipes where half repeat
    ONE id into ONE key (one register word takes a million racing updates)
    and the rest spread over 40k keys; registers == the oracle."""
    from rtsas_amd.engine import DeviceBatch, DeviceBuffer
    w, p = _c3_small(engine)
    engine.hll_reserve(40_001)
    b = engine.swipe_batch(p, 0, 2_000_000)
    buf, offs, slot = b.to_host()
    slot = (np.arange(b.n, dtype=np.uint64) * 2654435761 % 40_000).astype(np.uint32)
    hot = np.arange(0, b.n, 2)
    first = bytes(buf[offs[0]:offs[1]])
    assert all(offs[i + 1] - offs[i] == 8 for i in (0, 1))
    ids = buf[:offs[-1]].reshape(-1, 8).copy()
    ids[hot] = np.frombuffer(first, np.uint8)
    slot[hot] = 40_000
    buf2 = np.concatenate([ids.reshape(-1), np.zeros(16, np.uint8)])
    d = DeviceBatch.from_host(engine.ctx, buf2, offs, slot)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, d, out)
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    regs = np.zeros((40_001, 16384), np.uint8)
    want, _, _ = orc.process_swipes(chain, regs, slot, buf2, offs)
    assert np.array_equal(out.to_host(np.uint8, b.n), want)
    assert np.array_equal(engine.registers_all(40_001), regs)


@pytest.mark.parametrize("mode", ["direct", "graph"])
def test_many_small_units(engine, orc, mode):
    """ske_swipes_many_async through the partitioned K1 with sub-batches of
    64k swipes: ~25 units over 7 ragged batches (incl. 1 swipe and a partial
    tile) reuse one scratch set in stream order, launched directly or
    replayed from a graph; answers and registers == the oracle over the
    batches in order."""
    import torch
    from rtsas_amd.engine import DeviceBuffer
    w, p = _c3_small(engine)
    engine.set_option("part_sub", 65536)
    sizes = [300_000, 1, 70_001, 300_000, 250_000, 2048, 400_000]
    bs, start = [], 0
    for n in sizes:
        bs.append(engine.swipe_batch(p, start, n))
        start += n
    outs = [DeviceBuffer(engine.ctx, b.n) for b in bs]
    main = torch.cuda.Stream()
    engine.set_stream(main.cuda_stream)
    try:
        if mode == "direct":
            engine.swipes_many_async(0, bs, outs)
        else:
            engine.swipes_many_async(0, bs[:2], outs[:2])  # scratch sized before the capture
            torch.cuda.synchronize()
            g = engine.capture(lambda: engine.swipes_many_async(0, bs, outs))
            g.launch()
        engine.sync()
        if mode == "graph":
            g.free()
    finally:
        engine.set_stream(None)
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    for b, o in zip(bs, outs):
        buf, offs, slot = b.to_host()
        v, _, _ = orc.process_swipes(chain, regs, slot.astype(np.uint32), buf, offs)
        assert np.array_equal(o.to_host(np.uint8, b.n), v)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


def test_host_staged_large_batch_equals_device_resident(engine, orc):
    """A 3M-swipe batch handed over in pageable host memory (SKE_MEM_HOST) is
    staged through the library's pinned double buffer by its copy threads
    (inputs above 8 MB, several 32 MB chunks); answers and registers equal the
    same batch run device-resident.  Offsets that decrease inside a later
    chunk are refused (SKE_EINVAL) with the registers untouched."""
    import ctypes as C
    from rtsas_amd._lib import SKE_EINVAL, SKE_MEM_HOST
    from rtsas_amd.engine import DeviceBuffer
    from rtsas_amd import SketchLibError
    w, p = _c3_small(engine)
    n = 3_000_000
    b = engine.swipe_batch(p, 0, n)
    buf, offs, slot = b.to_host()
    buf = np.concatenate([buf, np.zeros(16, np.uint8)])
    assert buf.nbytes > (8 << 20) and offs.nbytes > (8 << 20)
    ptr = lambda a: C.c_void_p(a.ctypes.data)
    bad = offs.copy()
    k = 2_500_000                      # inside the second 32 MB chunk of the bytes, late in the offsets
    bad[k], bad[k + 1] = bad[k + 1], bad[k]
    out = np.zeros(n, np.uint8)
    with pytest.raises(SketchLibError) as ei:
        engine.ctx.call("ske_swipes", 0, ptr(slot), ptr(buf), ptr(bad), n, ptr(out), SKE_MEM_HOST)
    assert ei.value.code == SKE_EINVAL
    assert not engine.registers_all(w.n_keys).any()
    engine.ctx.call("ske_swipes", 0, ptr(slot), ptr(buf), ptr(offs), n, ptr(out), SKE_MEM_HOST)
    host_regs = engine.registers_all(w.n_keys).copy()
    engine.hll_reserve(2 * w.n_keys)
    b.slot.from_host(slot + w.n_keys)
    dout = DeviceBuffer(engine.ctx, n)
    engine.swipes(0, b, dout)
    assert np.array_equal(out, dout.to_host(np.uint8, n))
    assert np.array_equal(engine.registers_all(2 * w.n_keys)[w.n_keys:], host_regs)
    assert out.sum() > 0.8 * n


@pytest.mark.parametrize("mem", ["host", "device"])
def test_fixed_bits_feed_equals_device_resident(pkg, engine, orc, mem):
    """ske_swipes_fixed_bits: fixed-width ids, answers 1 bit per swipe, host
    batches pipelined in 4M-swipe chunks (copy stream beside K1).  Over 9M + 5
    swipes (three chunks, a ragged last byte) on the C3 filter its answers and
    registers equal the device-resident ske_swipes of the same batch on
    another context, and the oracle's on a sample."""
    import ctypes as C
    from rtsas_amd import synthetic
    from rtsas_amd._lib import SKE_MEM_DEVICE, SKE_MEM_HOST
    from rtsas_amd.engine import DeviceBuffer, SketchEngine
    w = synthetic.WORKLOADS["c3"]
    w = synthetic.Workload(**{**w.__dict__, "n_members": 300_000, "n_keys": 500, "zipf_lectures": 0,
                              "zipf_days": 0})
    n = 9 * 1024 * 1024 + 5
    engines = [engine, SketchEngine(0)]
    for e in engines:
        e.reserve(0, w.bf_error, w.bf_capacity)
        p = e.gen_params(w)
        e.preload(0, p, w.n_members)
        e.hll_reserve(w.n_keys)
        assert e.variant(0) == 3
    ref, fed = engines
    b = ref.swipe_batch(ref.gen_params(w), 0, n)
    out = DeviceBuffer(ref.ctx, n)
    ref.swipes(0, b, out)
    want = out.to_host(np.uint8, n)
    buf, offs, slot = b.to_host()
    width = int(offs[1] - offs[0])
    ids = np.ascontiguousarray(buf[:n * width].reshape(n, width))
    bits = np.zeros((n + 7) // 8, np.uint8)
    if mem == "host":
        fed.ctx.call("ske_swipes_fixed_bits", 0, slot.ctypes.data_as(C.c_void_p), ids.ctypes.data_as(C.c_void_p), width, n,
                     bits.ctypes.data_as(C.c_void_p), SKE_MEM_HOST)
    else:
        fb = fed.swipe_batch(fed.gen_params(w), 0, n)
        dbits = DeviceBuffer(fed.ctx, bits.size)
        fed.ctx.call("ske_swipes_fixed_bits", 0, C.c_void_p(fb.slot.ptr), C.c_void_p(fb.bytes.ptr), width, n,
                     C.c_void_p(dbits.ptr), SKE_MEM_DEVICE)
        bits = dbits.to_host(np.uint8, bits.size)
    got = np.unpackbits(bits, count=n, bitorder="little")
    assert np.array_equal(got, want)
    assert np.array_equal(fed.registers_all(w.n_keys), ref.registers_all(w.n_keys))
    # the oracle on the first 200k swipes (answers depend on the Bloom only)
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = ref.members_batch(ref.gen_params(w), 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    k = 200_000
    v, _ = chain.mexists_packed(buf[:k * width + 16], offs[:k + 1])
    assert np.array_equal(got[:k], v)


def test_client_swipes_fixed(client, orc):
    """SketchClient.swipes_fixed (the facade's fixed-width, bit-packed form)
    == swipes_slots == the oracle."""
    rng = np.random.default_rng(5)
    members = rng.choice(np.arange(10_000_000, 99_999_999), 50_000, replace=False)
    client.execute_command("BF.RESERVE", "bf", 0.001, 10_000_000)
    from rtsas_amd import pack_ints
    client.bf_madd_packed("bf", *pack_ints(members))
    ids = np.where(rng.random(300_001) < 0.9, rng.choice(members, 300_001), rng.integers(10**7, 10**8, 300_001))
    keys = [f"hll:unique:L{k}:2025-10-03" for k in range(9)]
    slots = np.asarray([client.key_slot(k) for k in keys], np.uint32)[rng.integers(0, 9, ids.size)]
    buf, offs = pack_ints(ids)
    fixed = buf.reshape(-1, 8)
    got = client.swipes_fixed("bf", slots, fixed)
    chain = orc.Chain(10_000_000, 0.001)
    chain.madd_packed(*pack_ints(members))
    want, _ = chain.mexists_packed(np.concatenate([buf, np.zeros(16, np.uint8)]), offs)
    assert np.array_equal(got, want.astype(bool))
    regs = [client.hll_registers(k) for k in keys]
    assert np.array_equal(client.swipes_slots("bf", slots, buf, offs), got)   # replay: same answers
    assert all(np.array_equal(client.hll_registers(k), r) for k, r in zip(keys, regs))   # idempotent
