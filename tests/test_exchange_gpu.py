"""Unpartitioned swipes routed by alltoallv on the device path (SURVEY.md
§8e): W ranks on this box's GPU (gloo transport; RCCL on a node), each with
its own slice of the stream over global key indices of a named universe.
distributed.SwipeExchange sends every swipe to its key's owner (distributed.
KeyMap), K1 runs there, the answers come back in the input order; then
distributed.ShardedSketch answers union PFCOUNT, PFCOUNT of every key and a
rollup by key NAME.  Answers == the oracle's BF.EXISTS; every rank's
registers == the single-process registers of the keys it owns; the
cluster-wide queries == the one-shard oracle."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,mode,backend", [(2, "exact", "gloo"), (3, "exact", "gloo"), (2, "async", "gloo"),
                                                (3, "async", "gloo"), (2, "async_overflow", "gloo"),
                                                (3, "async_many", "gloo"), (2, "async_serial", "gloo"),
                                                (1, "exact", "nccl"), (1, "async", "nccl"),
                                                (1, "async_many", "nccl")])
def test_exchange_on_device_equals_oracle(orc, engine, tmp_path, world, mode, backend):
    """mode exact: SwipeExchange.swipes (the host reads the routing counts);
    async: swipes_async over two batches (ske_route_swipes_cap_async, equal
    splits of a capacity that cannot overflow, padding into each rank's sink
    slot) then settle(), in the pipelined form (batch j+1's routing and
    forward exchange on their own stream beside batch j's K1, two parities
    of rows); async_many: five batches (each parity reused); async_serial:
    the one-stream form; async_overflow: a capacity below the owners' shares,
    so settle() re-runs both batches with exact splits.  backend nccl: RCCL
    (one GPU holds one RCCL rank: world 1, with the collectives forced on --
    the device all_to_all_single / all_reduce / reduce_scatter_tensor /
    all_gather calls of a multi-GPU node, on their RCCL code path)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from exchange_worker import NK, groups, names, workload
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", WORKER_BACKEND=backend,
               WORKER_FORCE_COLLECTIVES="1" if backend == "nccl" else "0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
                        "--master-port", str(29650 + world + (10 if backend == "nccl" else 0)),
                        os.path.join(ROOT, "tests", "exchange_worker.py"),
                        str(tmp_path), mode], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[:4000] + r.stderr[-1500:]
    w = workload()
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    chain.madd_packed(mb[0], mb[1])
    regs = np.zeros((NK, 16384), np.uint8)
    for rk in range(world):
        d = np.load(tmp_path / f"r{rk}.npz")
        want, _, _ = orc.process_swipes(chain, regs, d["slot"].astype(np.uint32), d["buf"], d["offs"])
        assert np.array_equal(d["ans"], want.astype(np.uint8)), f"rank {rk} answers"
    seen = 0
    for rk in range(world):
        d = np.load(tmp_path / f"r{rk}.npz")
        for j, g in enumerate(d["mine"]):
            assert np.array_equal(d["regs"][j], regs[g]), f"key {g} on rank {rk}"
        seen += len(d["mine"])
        nm = names()
        idx = {n: i for i, n in enumerate(nm)}
        assert int(d["union"][0]) == orc.hll_count_regs(regs.max(axis=0))
        assert d["each"].tolist() == [orc.hll_count_regs(regs[g]) for g in range(NK)]
        assert d["roll"].tolist() == [orc.hll_count_regs(regs[[idx[n] for n in g]].max(axis=0)) if g else 0
                                      for g in groups(nm)]
    assert seen == NK



@pytest.mark.parametrize("slack,world", [(0.2, 2), (-0.6, 2), (0.1, 3), (-0.5, 5)])
def test_route_cap_layout(engine, slack, world):
    """ske_route_swipes_cap_async alone (one process, no collective): owner
    o's swipes fill rows [o*cap, o*cap + min(count_o, cap)) with their ids
    and local slots, owner o's other rows are padding (zero ids, sink[o]),
    pos[i] is a row of swipe i's owner holding swipe i (or, past cap, another
    swipe of that owner), counts are the owners' counts -- also with
    capacities below the owners' shares (slack < 0)."""
    import torch
    from rtsas_amd.distributed import NO_SLOT, KeyMap, SwipeExchange
    names = [f"hll:unique:L{k:03d}:2025-01-01" for k in range(37)]
    km = KeyMap(names, world)
    sinks = [km.slots_end(r) for r in range(world)]
    ex = SwipeExchange(0, world, None, km, engine=engine, sink_slots=sinks, slack=slack)
    rng = np.random.default_rng(3)
    cap = ex.capacity(200_000)
    for n in (200_000, 199_000, 1):
        idn = rng.integers(48, 58, (n, 8), dtype=np.uint8)
        # global keys -1 and 37..39 are outside the universe: rank 0, slot NO_SLOT
        gk = rng.integers(-1, 40, n)
        send_ids, send_slots, pos, counts = ex._route_cap_native(torch.from_numpy(idn).cuda(),
                                                                 torch.from_numpy(gk).cuda(), cap)
        torch.cuda.synchronize()
        sid, ssl = send_ids.cpu().numpy(), send_slots.cpu().numpy().view(np.uint32)
        ps, ct = pos.cpu().numpy()[:n].astype(np.int64), counts.cpu().numpy()
        known = (gk >= 0) & (gk < 37)
        gc = np.where(known, gk, 0)
        own = np.where(known, km.owner[gc], 0).astype(np.int64)
        loc = np.where(known, km.local[gc], NO_SLOT).astype(np.uint32)
        assert ct.tolist() == np.bincount(own, minlength=world).tolist()
        assert ((ps // cap) == own).all()
        for o in range(world):
            k = min(int(ct[o]), cap)
            rows = o * cap + np.arange(cap)
            hit = np.zeros(cap, bool)
            hit[ps[own == o] - o * cap] = True
            assert hit[:k].all() and not hit[k:].any()
            assert (ssl[rows[k:]] == sinks[o]).all() and not sid[rows[k:]].any()
        # every real row holds (the id, the local slot) of one of the swipes that name it
        def key(row, slot, id64):
            return (row.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ (slot.astype(np.uint64) << np.uint64(40)) \
                ^ id64
        want = key(ps, loc, idn.view(np.uint64).ravel())
        rr = np.unique(ps)
        have = key(rr, ssl[rr], sid.view(np.uint64).ravel()[rr])
        assert np.isin(have, want).all()


@pytest.mark.parametrize("padded,base", [(True, 0), (False, 0), (True, 2)])
def test_solo_exchange_identity_vs_oracle(orc, engine, padded, base):
    """World 1 without a process group: SwipeExchange.swipes_async is the
    identity -- keys mapped to local slots by ske_route_slots_async (base 0:
    the identity table, no gather; base 2: the key map's route table), K1 on
    the ids in place (padded: their storage has bytes past the last id; else
    they are copied into a padded buffer first), answers in input order over
    3 ragged batches; a global key past the universe gets its BF.EXISTS
    answer, its PFADD dropped and reported as SKE_ERANGE.  Answers and
    registers == the oracle."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from exchange_worker import NK, names, workload
    from rtsas_amd._lib import SketchLibError, SKE_ERANGE
    from rtsas_amd.distributed import KeyMap, SwipeExchange, engine_k1
    w = workload()
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    engine.preload(0, p, w.n_members)
    km = KeyMap(names(), 1, base=base)
    assert km.identity == (base == 0)
    engine.hll_reserve(base + NK + 1)
    ex = SwipeExchange(0, 1, engine_k1(engine), km, engine=engine, sink_slots=[base + NK])
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    mb = engine.members_batch(p, 0, w.n_members).to_host()
    chain.madd_packed(mb[0], mb[1])
    regs = np.zeros((base + NK + 1, 16384), np.uint8)
    start, outs, want = 0, [], []
    for j, n in enumerate([100_003, 1, 77_777]):
        buf, offs, slot = engine.swipe_batch(p, start, n).to_host()
        start += n
        width = int(offs[1] - offs[0])
        raw = np.zeros(n * width + (64 if padded else 0), np.uint8)
        raw[:n * width] = buf[:n * width]
        ids = torch.from_numpy(raw).cuda()[:n * width].view(n, width)
        g = slot.astype(np.int64)
        if j == 2:
            g[4321] = NK + 5  # past the universe
        outs.append(ex.swipes_async(ids, torch.from_numpy(g).cuda()))
        sl = slot.astype(np.uint32) + np.uint32(base)
        if j == 2:
            sl[4321] = base + NK  # the oracle's spare row (not compared)
        v, _, _ = orc.process_swipes(chain, regs, sl, buf, offs)
        want.append(v)
    assert ex.settle() == 0
    torch.cuda.synchronize()
    with pytest.raises(SketchLibError) as ei:
        engine.check_errors()
    assert ei.value.code == SKE_ERANGE
    for o, v in zip(outs, want):
        assert np.array_equal(o.cpu().numpy(), v.astype(np.uint8))
    assert np.array_equal(engine.registers_all(base + NK), regs[:base + NK])
