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


@pytest.mark.parametrize("world,mode", [(2, "exact"), (3, "exact"), (2, "async"), (3, "async"),
                                        (2, "async_overflow")])
def test_exchange_on_device_equals_oracle(orc, engine, tmp_path, world, mode):
    """mode exact: SwipeExchange.swipes (the host reads the routing counts);
    async: swipes_async over two batches (ske_route_swipes_cap_async, equal
    splits of a capacity that cannot overflow, padding into each rank's sink
    slot) then settle(); async_overflow: a capacity below the owners' shares,
    so settle() re-runs both batches with exact splits."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from exchange_worker import NK, groups, names, workload
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
                        "--master-port", str(29650 + world), os.path.join(ROOT, "tests", "exchange_worker.py"),
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
