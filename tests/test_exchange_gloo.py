"""Unpartitioned input: distributed.SwipeExchange routes each
rank's swipes to their key owners with all_to_all_single (alltoallv) and
returns the answers in the input order.  world_size 2 and 3 on gloo / CPU
tensors; K1 is replaced by the CPU oracle per rank (test infrastructure);
the routing, the splits and the un-permutation are the product code under
test.  Answers == BF.EXISTS of every swipe; each rank's registers == the
single-process registers of the keys it owns (slot s -> rank s % world,
local slot s // world)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NKEYS, N, W = 11, 3000, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _members():
    return [str(10_000_000 + 7 * i).encode() for i in range(500)]


def _stream(rank):
    rng = np.random.default_rng(100 + rank)
    mem = _members()
    ids = [mem[int(j)] if rng.random() < 0.8 else str(int(rng.integers(20_000_000, 99_999_999))).encode()
           for j in rng.integers(0, len(mem), N - rank * 7)]   # uneven sizes per rank
    buf = np.frombuffer(b"".join(ids), np.uint8).reshape(-1, W).copy()
    # a skewed key distribution (hot low slots), global slots
    slots = np.minimum(rng.zipf(1.5, len(ids)) - 1, NKEYS - 1).astype(np.int64)
    return buf, slots


def _chain(orc):
    ch = orc.Chain(1000, 0.01)
    mem = _members()
    buf = np.frombuffer(b"".join(mem) + b"\0" * 16, np.uint8).copy()
    offs = np.arange(0, W * len(mem) + 1, W, dtype=np.uint32)
    ch.madd_packed(buf, offs)
    return ch


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    ge.load_package()
    orc = ge.load_oracle()
    from rtsas_amd.distributed import SwipeExchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    chain = _chain(orc)
    nlocal = -(-NKEYS // world)
    regs = np.zeros((nlocal, 16384), np.uint8)

    def k1(ids, local_slots):   # the oracle as this rank's K1
        m = ids.shape[0]
        buf = np.concatenate([ids.numpy().reshape(-1), np.zeros(16, np.uint8)])
        offs = np.arange(0, W * m + 1, W, dtype=np.uint32)
        v, _, _ = orc.process_swipes(chain, regs, local_slots.numpy().astype(np.uint32), buf, offs)
        return torch.from_numpy(v.astype(np.uint8))

    ex = SwipeExchange(rank, world, k1)
    buf, slots = _stream(rank)
    ans = ex.swipes(torch.from_numpy(buf), torch.from_numpy(slots))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), ans=ans.numpy(), regs=regs)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_equals_owner_routing(orc, tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    chain = _chain(orc)
    regs = np.zeros((NKEYS, 16384), np.uint8)
    for r in range(world):   # the single-process run over every rank's stream
        buf, slots = _stream(r)
        flat = np.concatenate([buf.reshape(-1), np.zeros(16, np.uint8)])
        offs = np.arange(0, W * len(slots) + 1, W, dtype=np.uint32)
        want, _, _ = orc.process_swipes(chain, regs, slots.astype(np.uint32), flat, offs)
        got = np.load(tmp_path / f"r{r}.npz")["ans"]
        assert np.array_equal(got, want.astype(np.uint8)), f"rank {r} answers"
    assert regs.any()
    for s in range(NKEYS):
        rr = np.load(tmp_path / f"r{s % world}.npz")["regs"]
        assert np.array_equal(rr[s // world], regs[s]), f"slot {s}"
