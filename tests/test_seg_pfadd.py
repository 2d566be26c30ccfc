"""The segmented PFADD (sketch_part.hip k_seg_c1 / k_seg_da (or k_seg_scan + k_seg_d) /
k_seg_e): pass C of the one-link partitioned K1 when a batch's register
updates are dense in the slab -- valid swipes' (register, rank) records
bucketed by key, each window of keys staged in LDS, raised there and its
risen lines stored back.  The result must equal the sequential hllAdd()s of
attendance_processor.py:127-129 (max is commutative) and the answers the
BF.EXISTS of :109-113, bit-exact against the oracle
(oracle/sketch_oracle.c).

Covered: forced on (option hll_seg = 1) on small C3-geometry streams with
Zipf-skewed keys, windows of 4 and 8 keys, every window staged in LDS
(seg_dense_min 0), none staged (raised in place), the default mix; several
sub-batches feeding one window pass (part_sub); key counts that are not a
multiple of the window; an out-of-range slot (error channel); ragged ids of
0..40 bytes; the auto choice (a 1.6 MB slab at its threshold, and the
8-way shard's 12 500 keys: pass C at a 16 M-swipe batch, this form at the
2^27 step); graph capture; and C3 at the bench's sizes in test_full_size.py
(the N = 1 default step and the 8-way shard's 2^27 step auto-select this
form).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _c3(engine, n_members=200_000, lectures=37, days=10):
    from rtsas_amd import synthetic
    w = synthetic.WORKLOADS["c3"]
    w = synthetic.Workload(**{**w.__dict__, "n_members": n_members, "n_keys": lectures * days,
                              "zipf_lectures": lectures, "zipf_days": days})
    engine.reserve(0, w.bf_error, w.bf_capacity)   # the 19.8 MB C3 geometry (one link, k = 11)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    assert engine.variant(0) == 3
    return w, p


def _oracle(orc, engine, w, p, batches):
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members)
    buf, offs, _ = mb.to_host()
    mb.free()
    chain.madd_packed(buf, offs)
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    answers = []
    for b in batches:
        buf, offs, slot = b.to_host()
        v, _, _ = orc.process_swipes(chain, regs, slot.astype(np.uint32), buf, offs)
        answers.append(v)
    return chain, regs, answers


@pytest.mark.parametrize("klog,dense_min,sub", [
    (3, 100, 0),            # default mix of staged and in-place windows
    (3, 0, 0),              # every window with records staged in LDS
    (3, 10 ** 6, 0),        # no window staged: every record raised in place
    (2, 100, 0),            # windows of 4 keys (two blocks per CU)
    (3, 0, 1 << 18),        # 5 sub-batches feed one window pass
    (2, 50, 3 * 1024 + 5),  # sub-batches of 4 tiles (rounded), odd split
    (1, 100, 0),            # windows of 2 keys (512-thread blocks)
    (0, 100, 0),            # windows of 1 key (256-thread blocks)
    (0, 0, 1 << 18),        # 1-key windows, 5 sub-batches, all staged
    (1, 100, 16384),        # 74 sub-batches: two window passes (64 + 10 sub-batches)
])
def test_seg_forced_small(engine, orc, klog, dense_min, sub):
    from rtsas_amd.engine import DeviceBuffer
    w, p = _c3(engine, lectures=37, days=10)   # 370 keys: not a multiple of 4 or 8 windows
    engine.set_option("hll_seg", 1)
    engine.set_option("seg_klog", klog)
    engine.set_option("seg_dense_min", dense_min)
    if sub:
        engine.set_option("part_sub", sub)
    n = 1_200_000 + 77  # a ragged last tile and run
    b = engine.swipe_batch(p, 0, n)
    out = DeviceBuffer(engine.ctx, n)
    engine.swipes(0, b, out)
    _, regs, answers = _oracle(orc, engine, w, p, [b])
    assert np.array_equal(out.to_host(np.uint8, n), answers[0])
    assert np.array_equal(engine.registers_all(w.n_keys), regs)
    # a second batch onto the risen registers (the dirty-line write-back)
    b2 = engine.swipe_batch(p, n, n)
    engine.swipes(0, b2, out)
    _, regs, answers = _oracle(orc, engine, w, p, [b, b2])
    assert np.array_equal(out.to_host(np.uint8, n), answers[1])
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


@pytest.mark.parametrize("nkeys,n,klog", [(1, 700_001, 3), (9, 700_001, 3), (4097, 700_001, 3),
                                           (20_000, 700_001, 3), (1, 12_000_000, 2), (3, 9_000_000, 3),
                                           (20_000, 700_001, 0), (3, 9_000_000, 0), (4097, 700_001, 1)])
def test_seg_key_counts(engine, orc, nkeys, n, klog):
    """Slabs of 1 key (one bucket, one window), 9 (a partial window), 4097
    (a partial last bucket) and 20 000 (512-bucket cap: s1 grows), uniform
    keys, forced on; one key under 12 M swipes (a window of > 1024 runs --
    staged in batches -- cut into ~165 slices), three under 9 M."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c3"]
    w = synthetic.Workload(**{**w.__dict__, "n_members": 100_000, "n_keys": nkeys,
                              "zipf_lectures": 0, "zipf_days": 0})
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    engine.set_option("hll_seg", 1)
    engine.set_option("seg_klog", klog)
    b = engine.swipe_batch(p, 0, n)
    out = DeviceBuffer(engine.ctx, n)
    engine.swipes(0, b, out)
    _, regs, answers = _oracle(orc, engine, w, p, [b])
    assert np.array_equal(out.to_host(np.uint8, n), answers[0])
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


@pytest.mark.parametrize("nkeys,klog", [(4097, 1), (20_000, 3), (300, 0)])
def test_seg_all_valid_runs(engine, orc, nkeys, klog):
    """Every swipe valid (no invalid ids): a full C1 run holds 8192 records,
    so the arena form's 4-record pads no longer fit its LDS and it takes the
    unpadded layout, storing each bucket's pad itself (k_seg_c1)."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c3"]
    w = synthetic.Workload(**{**w.__dict__, "n_members": 100_000, "n_keys": nkeys, "invalid_frac": 0.0,
                              "zipf_lectures": 0, "zipf_days": 0})
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    engine.set_option("hll_seg", 1)
    engine.set_option("seg_klog", klog)
    n = 900_001
    b = engine.swipe_batch(p, 0, n)
    out = DeviceBuffer(engine.ctx, n)
    engine.swipes(0, b, out)
    _, regs, answers = _oracle(orc, engine, w, p, [b])
    assert answers[0].all()
    assert np.array_equal(out.to_host(np.uint8, n), answers[0])
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


def _rand_items(rng, n, maxlen, minlen=0):
    lens = rng.integers(minlen, maxlen + 1, n)
    return [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]


def _pack(items):
    offs = np.zeros(len(items) + 1, np.uint32)
    offs[1:] = np.cumsum([len(x) for x in items])
    buf = np.frombuffer(b"".join(items) + b"\0" * 16, np.uint8).copy()
    return buf, offs


def test_seg_ragged_ids_hot_key(engine, orc):
    """0..40-byte ids (pass A's generic hash), one key taking 60 % of the
    swipes (a bucket whose runs fill whole chunks), C3's one-link filter.
    In the arena form the hot key's bucket holds ~12 chunks against kstat = 6
    fixed slots per bucket (16 buckets, 22 chunks): its later chunks take
    counted slots through the chunk table."""
    import ctypes as C
    from rtsas_amd.engine import DeviceBatch, DeviceBuffer
    rng = np.random.default_rng(5)
    members = _rand_items(rng, 40000, 40, 1)
    engine.reserve(0, 0.001, 10_000_000)
    mb, mo = _pack(members)
    dm = DeviceBatch.from_host(engine.ctx, mb, mo, np.zeros(len(members), np.uint32))
    engine.ctx.call("ske_bf_madd", 0, C.c_void_p(dm.bytes.ptr), C.c_void_p(dm.offs.ptr), len(members), None, 1)
    chain = orc.Chain(10_000_000, 0.001)
    chain.madd_packed(mb, mo)
    items = [members[int(i)] for i in rng.integers(0, len(members), 150000)]
    items += _rand_items(rng, 30000, 40) + [b""] * 40
    items = [items[int(i)] for i in rng.permutation(len(items))]
    nk = 300
    keys = np.where(rng.random(len(items)) < 0.6, 17, rng.integers(0, nk, len(items))).astype(np.uint32)
    buf, offs = _pack(items)
    engine.hll_reserve(nk)
    engine.set_option("hll_seg", 1)
    b = DeviceBatch.from_host(engine.ctx, buf, offs, keys)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    regs = np.zeros((nk, 16384), np.uint8)
    valid, _, _ = orc.process_swipes(chain, regs, keys, buf, offs)
    assert np.array_equal(out.to_host(np.uint8, b.n), valid)
    assert np.array_equal(engine.registers_all(nk), regs)


def test_seg_out_of_range_slot(engine, orc):
    """A valid swipe naming a slot past the slab: SKE_ERANGE from the
    synchronous call, its answer still written, no register touched, the
    other swipes exact."""
    from rtsas_amd._lib import SketchLibError, SKE_ERANGE
    from rtsas_amd.engine import DeviceBatch, DeviceBuffer
    w, p = _c3(engine, lectures=10, days=10)
    engine.set_option("hll_seg", 1)
    n = 300_000
    b = engine.swipe_batch(p, 0, n)
    buf, offs, slot = b.to_host()
    slot = slot.astype(np.uint32)
    slot[::1000] = w.n_keys + 5  # outside the slab
    bb = DeviceBatch.from_host(engine.ctx, buf, offs, slot)
    out = DeviceBuffer(engine.ctx, n)
    with pytest.raises(SketchLibError) as ei:
        engine.swipes(0, bb, out)
    assert ei.value.code == SKE_ERANGE
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members)
    mbuf, moffs, _ = mb.to_host()
    chain.madd_packed(mbuf, moffs)
    keep = slot < w.n_keys
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    sel = np.nonzero(keep)[0]
    width = int(offs[1] - offs[0])
    sb = np.ascontiguousarray(buf[:n * width].reshape(n, width)[sel]).reshape(-1)
    so = np.arange(0, width * sel.size + 1, width, dtype=np.uint32)
    orc.process_swipes(chain, regs, slot[sel], sb, so)
    allv = np.array([chain.exists(bytes(buf[offs[i]:offs[i + 1]])) for i in range(0, n, 1000)], np.uint8)
    got = out.to_host(np.uint8, n)
    assert np.array_equal(got[::1000], allv)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


def test_seg_auto_choice(engine):
    """auto (-1): segmented from seg_density / 100 swipes per 128-B slab
    line (default 6), twice that for a slab the Infinity Cache holds (this
    one: 100 keys, 1.6 MB, 12 800 lines -> 153 600 swipes); the choice is the
    library's, visible through the pass timing kinds."""
    from rtsas_amd.engine import DeviceBuffer
    w, p = _c3(engine, lectures=10, days=10)   # 100 keys = 12 800 lines
    out = DeviceBuffer(engine.ctx, 1 << 20)
    engine.set_option("pass_timing", 1)

    def seg_used(n):
        engine.pass_times(reset=True)
        engine.swipes(0, engine.swipe_batch(p, 0, n), out)
        pt = engine.pass_times(reset=True)
        assert pt[3][1] > 0
        return pt[5][1] > 0

    assert not seg_used(150_000) and seg_used(160_000)
    engine.set_option("seg_density", 100)  # 2 per line (x2 on chip): 25 600
    assert not seg_used(25_000) and seg_used(26_000)
    engine.set_option("hll_seg", 0)
    assert not seg_used(1 << 20)
    engine.set_option("hll_seg", 1)
    assert seg_used(1000)
    engine.set_option("pass_timing", 0)


def test_seg_auto_choice_shard(engine):
    """The auto choice where it matters: the 8-way shard's slab (12 500 keys,
    204.8 MB, inside the 256 MiB Infinity Cache: 12 swipes per line, i.e.
    19.2 M swipes) keeps pass C for a 16 M-swipe batch (the shard's round-4
    step, where pass C measured faster) and takes the segmented form at the
    bench's 2^27 step; the threshold sits exactly at 12 swipes per line."""
    w, p = _c3(engine, n_members=100_000, lectures=125, days=100)   # 12 500 keys
    out = DeviceBuffer_of(engine, 1 << 27)
    engine.set_option("pass_timing", 1)
    engine.set_option("hll_seg", -1)
    engine.set_option("seg_density", 600)

    def seg_used(n):
        engine.pass_times(reset=True)
        engine.swipes(0, engine.swipe_batch(p, 0, n), out)
        pt = engine.pass_times(reset=True)
        assert pt[3][1] > 0
        return pt[5][1] > 0

    assert not seg_used(1 << 24)
    assert not seg_used(19_100_000) and seg_used(19_300_000)
    assert seg_used(1 << 27)
    engine.set_option("pass_timing", 0)


def DeviceBuffer_of(engine, n):
    from rtsas_amd.engine import DeviceBuffer
    return DeviceBuffer(engine.ctx, n)


def test_seg_graph_replay(engine, orc):
    """Batches recorded into a HIP graph through the segmented form (its
    scratch sized before the capture), replayed: answers and registers
    exact."""
    from rtsas_amd.engine import DeviceBuffer
    w, p = _c3(engine, lectures=20, days=10)
    engine.set_option("hll_seg", 1)
    n = 400_000
    batches = [engine.swipe_batch(p, j * n, n) for j in range(3)]
    outs = [DeviceBuffer(engine.ctx, n) for _ in batches]
    engine.swipes(0, batches[0], outs[0])  # sizes the scratch
    g = engine.capture(lambda: [engine.swipes_async(0, b, o) for b, o in zip(batches, outs)])
    g.launch()
    engine.sync()
    g.free()
    _, regs, answers = _oracle(orc, engine, w, p, batches)
    for a, o in zip(answers, outs):
        assert np.array_equal(o.to_host(np.uint8, n), a)
    # batch 0 ran twice (direct, then in the graph): PFADD is idempotent
    assert np.array_equal(engine.registers_all(w.n_keys), regs)
