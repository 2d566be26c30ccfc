"""Parity at the benchmark's own sizes (BASELINE.json configs), bit-exact.

The C oracle finishes a whole bench step in seconds, so the configurations
bench.py measures are checked exactly, not only through properties:

- C2: the bench's workload (100k members, 50 keys, 1M-swipe steps), four
  steps recorded into a HIP graph and replayed as bench.py does;
- C4: the adversarial stream (50 % invalid, half of them near-collisions of
  members: one decimal digit changed), one 1M-swipe step;
- C3: one GPU's shard of the 8-GPU C3 run (10M-member filter of 19.8 MB,
  12.5k Zipf lecture-day keys), one 16M-swipe step through the
  partitioned K1 (and the XCD-partitioned one);
- C3 at one GPU of the driver's N=1 bench (100k keys), one 16M-swipe step.

Answers, every register array and the probe / valid counts must equal the
oracle's (attendance_processor.py:100-137 restated, oracle/sketch_oracle.c).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle(orc, engine, w, p, batches, nkeys):
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members)
    buf, offs, _ = mb.to_host()
    mb.free()
    chain.madd_packed(buf, offs)
    regs = np.zeros((nkeys, 16384), np.uint8)
    answers, probes, nvalid = [], 0, 0
    for b in batches:
        buf, offs, slot = b.to_host()
        v, nv, pr = orc.process_swipes(chain, regs, slot.astype(np.uint32), buf, offs)
        answers.append(v)
        probes += pr
        nvalid += nv
    return chain, regs, answers, probes, nvalid


def _setup(engine, w):
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(w.n_keys)
    return p


def test_c2_bench_steps_graph_replay(engine, orc):
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c2"]
    p = _setup(engine, w)
    n = w.step_swipes
    batches = [engine.swipe_batch(p, j * n, n) for j in range(4)]
    outs = [DeviceBuffer(engine.ctx, n) for _ in batches]
    g = engine.capture(lambda: [engine.swipes_async(0, b, o) for b, o in zip(batches, outs)])
    g.launch()
    engine.sync()
    g.free()
    _, regs, answers, probes, nvalid = _oracle(orc, engine, w, p, batches, w.n_keys)
    for a, o in zip(answers, outs):
        assert np.array_equal(o.to_host(np.uint8, n), a)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)
    stats = [engine.swipes_stats(0, b) for b in batches]
    assert (sum(s[0] for s in stats), sum(s[1] for s in stats)) == (probes, nvalid)
    assert 0.85 < nvalid / (4 * n) < 0.95


@pytest.mark.parametrize("variant", [-1, 3])
def test_c4_adversarial_step(engine, orc, variant):
    """C4 through the auto (LDS) K1 and the partitioned K1 forced onto its
    small filter: half the swipes non-members, half of those near-collisions,
    so pass B's fail lists overflow into fail bytes."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c4"]
    p = _setup(engine, w)
    engine.set_option("variant", variant)
    b = engine.swipe_batch(p, 0, w.step_swipes)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    _, regs, answers, probes, nvalid = _oracle(orc, engine, w, p, [b], w.n_keys)
    assert np.array_equal(out.to_host(np.uint8, b.n), answers[0])
    assert np.array_equal(engine.registers_all(w.n_keys), regs)
    assert engine.swipes_stats(0, b) == (probes, nvalid)
    # half the swipes are non-members; about 1 % of those pass the filter
    assert 0.49 < nvalid / b.n < 0.52


@pytest.mark.parametrize("variant", [-1, 2])
def test_c3_gpu_shard_full_step(engine, orc, variant):
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.shard(synthetic.WORKLOADS["c3"], 8)
    assert w.n_keys == 12_500 and w.step_swipes == 16_000_000
    p = _setup(engine, w)
    assert engine.variant(0) == 3  # partitioned K1 for the 19.8 MB filter
    engine.set_option("variant", variant)
    b = engine.swipe_batch(p, 0, w.step_swipes)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    chain, regs, answers, probes, nvalid = _oracle(orc, engine, w, p, [b], w.n_keys)
    assert np.array_equal(engine.bloom_bits(0, 0, chain.link_info(0)["bytes"]), chain.link_bits(0))
    assert np.array_equal(out.to_host(np.uint8, b.n), answers[0])
    assert np.array_equal(engine.registers_all(w.n_keys), regs)
    assert engine.swipes_stats(0, b) == (probes, nvalid)


@pytest.mark.parametrize("mode,branches", [("capture_branched", 4), ("native", 4),
                                           ("native-graph", 16), ("native-graph-fixed", 16),
                                           ("native-forked", 4), ("native-graph-forked", 16)])
def test_c2_bench_steps_forked_graph(engine, orc, mode, branches):
    """bench.py's timing.  native*: ske_swipes_many_async -- one persistent
    LDS K1 launch over all the steps (the default), or with k1_persistent = 0
    the steps on independent branches (step j on branch j mod B, two launches
    side by side on half the CUs), enqueued directly or recorded into a graph.
    capture_branched: torch streams, full-chip grid.  Concurrent launches
    update the same registers."""
    import functools
    import torch
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c2"]
    p = _setup(engine, w)
    n = w.step_swipes
    batches = [engine.swipe_batch(p, j * n, n) for j in range(2 * branches)]
    outs = [DeviceBuffer(engine.ctx, n) for _ in batches]
    fixed = mode.endswith("fixed")
    if mode.endswith("forked"):
        engine.set_option("k1_persistent", 0)
    main = torch.cuda.Stream()
    engine.set_stream(main.cuda_stream)
    try:
        if mode == "capture_branched":
            side = [torch.cuda.Stream() for _ in range(branches - 1)]
            steps = [functools.partial(engine.swipes_async, 0, b, o)
                     for b, o in zip(batches, outs)]
            g = engine.capture_branched(steps, main, side)
        elif mode in ("native", "native-forked"):
            g = None
            engine.swipes_many_async(0, batches, outs, branches=branches)
        else:
            engine.swipes_many_async(0, [], branches=branches)
            engine.swipes_many_async(0, batches[:1], outs[:1], branches=1, fixed=fixed)
            torch.cuda.synchronize()
            g = engine.capture(lambda: engine.swipes_many_async(
                0, batches[1:], outs[1:], branches=branches, fixed=fixed))
        if g is not None:
            g.launch()
        torch.cuda.synchronize()
        if g is not None:
            g.free()
    finally:
        engine.set_stream(None)
    _, regs, answers, probes, nvalid = _oracle(orc, engine, w, p, batches, w.n_keys)
    for a, o in zip(answers, outs):
        assert np.array_equal(o.to_host(np.uint8, n), a)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


class _Slice:
    """A batch view of the first n swipes of a DeviceBatch (n may be 0)."""
    def __init__(self, b, n):
        self.slot, self.bytes, self.offs, self.width, self.n = b.slot, b.bytes, b.offs, b.width, n


@pytest.mark.parametrize("mode", ["direct", "graph", "graph-fixed"])
def test_c2_persistent_many_ragged(engine, orc, mode):
    """The persistent LDS K1 (one launch over the batch array): 53 batches --
    more than one launch holds (48), so two launches -- of ragged sizes: empty,
    1, one tile +- 1 (2048 swipes at U = 2), and up to 200k; tiles never span
    batches and a block's share crosses many batch boundaries.  Answers and
    registers == the oracle over the batches in order."""
    import torch
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.WORKLOADS["c2"]
    p = _setup(engine, w)
    rng = np.random.default_rng(53)
    sizes = [0, 1, 2047, 2048, 2049, 0, 3] + rng.integers(1, 200_000, 46).tolist()
    full, views, start = [], [], 0
    for n in sizes:
        b = engine.swipe_batch(p, start, max(n, 1))
        start += max(n, 1)
        full.append(b)
        views.append(_Slice(b, n))
    outs = [DeviceBuffer(engine.ctx, max(n, 1)) for n in sizes]
    fixed = mode.endswith("fixed")
    main = torch.cuda.Stream()
    engine.set_stream(main.cuda_stream)
    try:
        if mode == "direct":
            engine.swipes_many_async(0, views, outs)
        else:
            g = engine.capture(lambda: engine.swipes_many_async(0, views, outs, fixed=fixed))
            g.launch()
        engine.sync()
        if mode != "direct":
            g.free()
    finally:
        engine.set_stream(None)
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    for b, n, o in zip(full, sizes, outs):
        if n == 0:
            continue
        buf, offs, slot = b.to_host()
        v, _, _ = orc.process_swipes(chain, regs, slot[:n].astype(np.uint32), buf, offs[:n + 1])
        assert np.array_equal(o.to_host(np.uint8, n), v)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


@pytest.mark.parametrize("variant", [-1, 2])
def test_c3_many_batches_graph(engine, orc, variant):
    """The partitioned (and XCD-partitioned) K1 through ske_swipes_many_async
    recorded into a graph, batches of different sizes: its launches share the
    context scratch (sized for the largest batch before the first launch), so
    each waits for the previous one across branches; answers and registers ==
    the oracle."""
    import torch
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.shard(synthetic.WORKLOADS["c3"], 8)
    p = _setup(engine, w)
    engine.set_option("variant", variant)
    assert engine.variant(0) == (3 if variant == -1 else 2)
    sizes = [1 << 21, 1 << 20, 3 << 20, 1 << 21]
    starts = np.cumsum([0] + sizes)
    batches = [engine.swipe_batch(p, int(s), n) for s, n in zip(starts, sizes)]
    outs = [DeviceBuffer(engine.ctx, b.n) for b in batches]
    main = torch.cuda.Stream()
    engine.set_stream(main.cuda_stream)
    try:
        engine.swipes_many_async(0, [], branches=4)
        # the first call sizes the scratch for the largest batch of the graph:
        # a capture cannot allocate (the recorded call would fail with EBUSY)
        engine.swipes_many_async(0, batches[:1], outs[:1], branches=1)
        torch.cuda.synchronize()
        from rtsas_amd._lib import SketchLibError, SKE_EBUSY
        if variant == -1:
            with pytest.raises(SketchLibError) as ei:
                engine.capture(lambda: engine.swipes_many_async(0, batches[1:], outs[1:],
                                                                branches=3))
            assert ei.value.code == SKE_EBUSY
            torch.cuda.synchronize()
        engine.swipes_many_async(0, batches[2:3], outs[2:3], branches=1)  # the largest
        torch.cuda.synchronize()
        g = engine.capture(lambda: engine.swipes_many_async(0, batches[1:], outs[1:],
                                                            branches=3))
        g.launch()
        torch.cuda.synchronize()
        g.free()
    finally:
        engine.set_stream(None)
    # batch 2 ran twice (sizing call + graph): registers are a max, answers equal
    _, regs, answers, probes, nvalid = _oracle(orc, engine, w, p, batches, w.n_keys)
    for a, o, b in zip(answers, outs, batches):
        assert np.array_equal(o.to_host(np.uint8, b.n), a)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)


def test_c3_bench_shard_one_gpu(engine, orc):
    """C3 as the driver's N=1 bench runs it (synthetic.shard(c3, 1): 100k
    Zipf lecture-day keys, a 1.6 GB slab), one 16M-swipe step through the
    partitioned K1, bit-exact vs the oracle on every answer and register."""
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.shard(synthetic.WORKLOADS["c3"], 1)
    assert w.n_keys == 100_000
    p = _setup(engine, w)
    assert engine.variant(0) == 3
    b = engine.swipe_batch(p, 0, w.step_swipes)
    out = DeviceBuffer(engine.ctx, b.n)
    engine.swipes(0, b, out)
    _, regs, answers, _, _ = _oracle(orc, engine, w, p, [b], w.n_keys)
    assert np.array_equal(out.to_host(np.uint8, b.n), answers[0])
    got = engine.registers_all(w.n_keys)
    assert np.array_equal(got, regs)


@pytest.mark.parametrize("world,n", [(1, 1 << 27), (8, 1 << 27), (1, 1 << 28)])
def test_c3_bench_step_128m_segmented(engine, orc, world, n):
    """C3 at bench.py's default steps: 2^27 swipes per GPU (round 5: a
    1B-swipe C3 stream in 8 steps) and 2^28 (round 6: in 4 steps, 8
    sub-batches feeding one window pass), on one GPU's keys at N = 1 (100k
    Zipf lecture-day keys, a 1.6 GB slab) and at N = 8
    (synthetic.shard(c3, 8): 12.5k keys, 205 MB).  The auto choice takes the
    segmented PFADD at this density (asserted through the pass timing kinds);
    every answer and every register bit-exact vs the oracle (its
    multi-threaded per-event loop, identical results to the sequential one).
    N = 1 in the default sub-batches (2^25 swipes), N = 8 in sub-batches of
    2^24."""
    import os
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    w = synthetic.shard(synthetic.WORKLOADS["c3"], world)
    p = _setup(engine, w)
    sub = 0 if world == 1 else 1 << 24
    engine.set_option("part_sub", sub)
    b = engine.swipe_batch(p, 0, n)
    out = DeviceBuffer(engine.ctx, n)
    engine.set_option("pass_timing", 1)
    engine.pass_times(reset=True)
    engine.swipes(0, b, out)
    pt = engine.pass_times(reset=True)
    engine.set_option("pass_timing", 0)
    nsub = n // ((1 << 25) if sub == 0 else sub)
    assert pt[5][1] == 1 and pt[4][1] == nsub, pt  # one window pass, nsub sub-batches
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members)
    mbuf, moffs, _ = mb.to_host()
    mb.free()
    chain.madd_packed(mbuf, moffs)
    buf, offs, slot = b.to_host()
    b.free()
    regs = np.zeros((w.n_keys, 16384), np.uint8)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    want, nvalid, _ = orc.process_swipes(chain, regs, slot.astype(np.uint32), buf, offs, threads=threads)
    del buf, offs, slot
    assert np.array_equal(out.to_host(np.uint8, n), want)
    assert np.array_equal(engine.registers_all(w.n_keys), regs)
    assert 0.85 < nvalid / n < 0.95
