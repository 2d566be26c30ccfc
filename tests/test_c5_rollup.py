"""C5 at its workload (BASELINE.json configs[4]): the campus-year slab of
365 days x 5000 lectures = 1.825M lecture-day HLL keys (30 GB) on one GPU,
filled by a 32M-swipe slice of the C5 stream through the partitioned K1, then
the PFCOUNT-form rankings of attendance_analysis.py:87-97 (README.md:179).

Checked against the oracle (oracle/sketch_oracle.c: Redis hllAdd / hllCount,
RedisBloom SBChain_Check), bit-exact:
- registers of a key sample -- every day of lecture 0 (the hottest, ~16 % of
  the stream), every day of lecture 7, and 300 random keys -- from only the
  swipes routed to those keys;
- per-lecture 365-key PFCOUNT unions (pfcount_groups) of lectures 0 and 7;
- PFCOUNT of every key (pfcount_each, the wave-per-key K2): the oracle
  estimator on the exported registers of the top / bottom-3 keys and of 200
  random keys, and top / bottom-3 == the first / last 3 of the full order;
- the campus-wide PFMERGE of all 1.825M keys (two-level K3) == the register
  max over the whole slab (torch amax on the device, an independent reduction).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_c5_campus_year_rollup(engine, orc):
    import torch
    from rtsas_amd import synthetic
    from rtsas_amd.processor import rank_top_bottom
    w = synthetic.WORKLOADS["c5"]
    nk = w.n_keys
    assert nk == 1_825_000
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    engine.hll_reserve(nk + 1)           # + the campus destination key
    assert engine.variant(0) == 3
    batches = [engine.swipe_batch(p, j * w.step_swipes, w.step_swipes) for j in range(2)]
    for b in batches:
        engine.swipes(0, b)
    # oracle: the chain, and the sampled keys' registers from their swipes only
    mb = engine.members_batch(p, 0, w.n_members)
    buf_m, offs_m, _ = mb.to_host()
    mb.free()
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    chain.madd_packed(buf_m, offs_m)
    rng = np.random.default_rng(5)
    days = w.zipf_days
    sample = np.unique(np.concatenate([np.arange(0, days), 7 * days + np.arange(days),
                                       rng.choice(nk, 300, replace=False)])).astype(np.uint32)
    index = np.full(nk, -1, np.int64)
    index[sample] = np.arange(len(sample))
    regs = np.zeros((len(sample), 16384), np.uint8)
    for b in batches:
        buf, offs, slot = b.to_host()
        sel = np.nonzero(index[slot] >= 0)[0]
        lens = (offs[sel + 1] - offs[sel]).astype(np.int64)
        assert (lens == 8).all()
        ids = buf[(offs[sel][:, None] + np.arange(8)).reshape(-1)]
        so = np.arange(0, 8 * len(sel) + 1, 8, dtype=np.uint32)
        orc.process_swipes(chain, regs, index[slot[sel]].astype(np.uint32), ids, so)
    for j, s in enumerate(sample):
        assert np.array_equal(engine.registers(int(s)), regs[j]), f"key {s}"
    # per-lecture unions of lectures 0 and 7
    slots = np.concatenate([np.arange(0, days), 7 * days + np.arange(days)]).astype(np.uint32)
    goffs = np.array([0, days, 2 * days], np.uint32)
    out = np.zeros(2, np.uint64)
    engine.ctx.call("ske_hll_pfcount_groups", slots.ctypes.data_as(C.c_void_p),
                    goffs.ctypes.data_as(C.c_void_p), 2, out.ctypes.data_as(C.c_void_p), 0)
    for g, lec in enumerate((0, 7)):
        u = regs[index[lec * days:(lec + 1) * days]].max(axis=0)
        assert int(out[g]) == orc.hll_count_regs(u)
    # PFCOUNT of every key, rankings
    counts = engine.pfcount_each(np.arange(nk, dtype=np.uint32)).astype(np.int64)
    names = [synthetic.key_name(w, k) for k in range(nk)]
    head, tail = rank_top_bottom(counts, names, 3)
    order_keys = np.lexsort((np.asarray(names), -counts))
    assert head == order_keys[:3].tolist() and tail == order_keys[-3:].tolist()
    check = np.unique(np.concatenate([head, tail, rng.choice(nk, 200, replace=False), sample]))
    for s in check:
        assert int(counts[s]) == orc.hll_count_regs(engine.registers(int(s))), f"key {s}"
    # campus-wide PFMERGE of every key into slot nk
    srcs = np.arange(nk, dtype=np.uint32)
    engine.ctx.call("ske_hll_pfmerge", nk, srcs.ctypes.data_as(C.c_void_p), nk)
    ptr, nbytes = C.c_void_p(), C.c_uint64()
    engine.ctx.call("ske_hll_slab", C.byref(ptr), C.byref(nbytes))

    class _Slab:  # zero-copy device view of the first nk keys of the slab
        __cuda_array_interface__ = {"shape": (nk, 16384), "typestr": "|u1", "data": (ptr.value, False),
                                    "version": 3, "strides": None}
    slab = torch.as_tensor(_Slab(), device="cuda")
    want = torch.amax(slab, dim=0).cpu().numpy()
    assert np.array_equal(engine.registers(nk), want)
    # the same queries device-resident end to end (round 6: plans on the GPU,
    # counts kept there, top / bottom-3 by torch.topk, PFMERGE over a device
    # source list) equal the host-staged ones above
    import rtsas_amd
    from rtsas_amd.distributed import KeyMap, ShardedSketch
    from rtsas_amd.processor import rank_top_bottom_dev
    client = rtsas_amd.SketchClient(context=engine.ctx)
    sk = ShardedSketch(client, 0, 1)
    km = KeyMap(names, 1)
    assert km.identity
    kp = sk.plan_keys(km, np.arange(nk))
    cdev = sk.pfcount_each_planned(kp)
    assert cdev.is_cuda and np.array_equal(cdev.cpu().numpy(), counts)
    assert rank_top_bottom_dev(cdev, 3) == (head, tail)  # names are in index order
    plan = sk.plan(km, [np.arange(0, days), 7 * days + np.arange(days)])
    assert sk.rollup_planned(plan, device=True).cpu().numpy().astype(np.uint64).tolist() == out.tolist()
    engine.ctx.call("ske_hll_clear", nk)
    campus, row = sk.pfmerge_planned(kp, nk)
    assert np.array_equal(row.cpu().numpy()[0], want) and campus == orc.hll_count_regs(want)
    # a device source list is range-checked on the device
    bad = torch.tensor([0, nk + 5, 3], dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(rtsas_amd.SketchLibError):
        engine.ctx.call("ske_hll_pfmerge_dev", nk, C.c_void_p(bad.data_ptr()), 3)
    with pytest.raises(rtsas_amd.SketchLibError):
        engine.ctx.call("ske_hll_pfcount_each", C.c_void_p(bad.data_ptr()), 3,
                        C.c_void_p(torch.zeros(3, dtype=torch.int64, device="cuda").data_ptr()), 1)
    for b in batches:
        b.free()
