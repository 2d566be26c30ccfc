"""Key-sharded sketch state across GPUs (one process per GPU).

The reference scales by running N processor processes on a Pulsar Shared
subscription (attendance_processor.py:30-34) against ONE Redis that
serialises every BF / PF op.  Here every GPU holds:

  * a replica of the Bloom chain (read-only on the hot path; preload is
    replayed on every rank -- BF.MADD is deterministic);
  * the HLL keys it owns: ``owner(key) = MurmurHash64A(key, 0) mod world``.

Swipes are routed to their key's owner at ingest (``route``), so the hot path
has no exchange.  Queries that span shards use one RCCL collective on u8
register arrays with MAX (HLL merge is an elementwise max, so the result is
bit-identical to a single-GPU run):

  * ``pfcount_union``  -- PFCOUNT k1 k2 ... across shards: local max-merge ->
    all_reduce(MAX) of 16 KiB -> K2 count;
  * ``rollup``         -- per-lecture unions over day keys spread over shards
    (config C5): local partial merges (G x 16 KiB) -> reduce_scatter(MAX) so
    each rank owns G/world lectures -> K2 counts -> all_gather of the counts
    (half the bytes of an all_reduce on the per-link-bound xGMI ring);
  * ``pfcount_each``   -- owner counts, one all_reduce(SUM) of u64 counts.

The device operations are behind a small ``ops`` object so the collective
logic runs unchanged with ``gloo`` on CPU tensors in the tests.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from .encoding import encode
from .keyhash import murmur64a

HLL_REGISTERS = 16384


def owner(key, world: int) -> int:
    return murmur64a(encode(key), 0) % world


def route(keys: Sequence, world: int) -> np.ndarray:
    """Owner rank of every key (ingest routing of swipes)."""
    cache: dict[bytes, int] = {}
    out = np.empty(len(keys), np.int32)
    for i, k in enumerate(keys):
        b = encode(k)
        r = cache.get(b)
        if r is None:
            r = cache[b] = murmur64a(b, 0) % world
        out[i] = r
    return out


class LibsketchOps:
    """Device side of the sharded queries (torch tensors on this rank's GPU)."""

    def __init__(self, client):
        import torch
        self.torch = torch
        self.client = client
        self.device = torch.device("cuda", client.ctx.device)

    def merge_groups(self, groups: Sequence[Sequence]) -> "torch.Tensor":
        t = self.torch.zeros((len(groups), HLL_REGISTERS), dtype=self.torch.uint8, device=self.device)
        slots, goffs = [], [0]
        for g in groups:
            for k in g:
                kb = encode(k)
                if self.client.keys.expect(kb, "hll"):
                    slots.append(self.client.keys.slot[kb])
            goffs.append(len(slots))
        if groups:
            self.torch.cuda.synchronize(self.device)
            s = np.asarray(slots or [0], np.uint32)
            go = np.asarray(goffs, np.uint32)
            self.client.ctx.call("ske_hll_merge_groups_dev", s.ctypes.data_as(C.c_void_p),
                                 go.ctypes.data_as(C.c_void_p), len(groups), C.c_void_p(t.data_ptr()))
        return t

    def count_raw(self, t) -> np.ndarray:
        out = np.zeros(t.shape[0], np.uint64)
        if t.shape[0]:
            self.torch.cuda.synchronize(self.device)
            self.client.ctx.call("ske_hll_count_raw_dev", C.c_void_p(t.data_ptr()), t.shape[0],
                                 out.ctypes.data_as(C.c_void_p))
        return out

    def count_each(self, keys: Sequence) -> np.ndarray:
        return self.client.pfcount_each(keys)


class ShardedSketch:
    def __init__(self, client, rank: int, world: int, group=None, ops=None):
        import torch.distributed as dist
        self.dist = dist
        self.client = client
        self.rank, self.world, self.group = rank, world, group
        self.ops = ops if ops is not None else LibsketchOps(client)
        backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
        self.use_reduce_scatter = backend == "nccl"

    def owns(self, key) -> bool:
        return owner(key, self.world) == self.rank

    def _max(self):
        return self.dist.ReduceOp.MAX

    def _all_reduce(self, t, op):
        """RCCL reduces device tensors in place; gloo (CPU tests, or ranks
        rehearsed on one GPU) gets a host copy of a device tensor."""
        if self.use_reduce_scatter or t.device.type == "cpu":
            self.dist.all_reduce(t, op=op, group=self.group)
            return t
        h = t.cpu()
        self.dist.all_reduce(h, op=op, group=self.group)
        t.copy_(h)
        return t

    def pfcount_union(self, keys: Sequence) -> int:
        mine = [k for k in keys if self.owns(k)]
        t = self.ops.merge_groups([mine])
        self._all_reduce(t, self._max())
        return int(self.ops.count_raw(t)[0])

    def pfcount_each(self, keys: Sequence) -> np.ndarray:
        import torch
        keys = list(keys)
        idx = [i for i, k in enumerate(keys) if self.owns(k)]
        counts = np.zeros(len(keys), np.int64)
        if idx:
            counts[idx] = self.ops.count_each([keys[i] for i in idx]).astype(np.int64)
        t = torch.from_numpy(counts)
        if self.use_reduce_scatter:
            t = t.to(self.ops.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t.cpu().numpy().astype(np.uint64)

    def rollup(self, groups: Sequence[Sequence]) -> np.ndarray:
        """Union count of every group of keys, keys anywhere in the cluster."""
        import torch
        G = len(groups)
        per = -(-G // self.world) if G else 0
        padded = [[k for k in g if self.owns(k)] for g in groups] + [[]] * (per * self.world - G)
        t = self.ops.merge_groups(padded)
        if self.use_reduce_scatter:
            mine = torch.empty((per, HLL_REGISTERS), dtype=t.dtype, device=t.device)
            self.dist.reduce_scatter_tensor(mine, t, op=self._max(), group=self.group)
        else:
            self._all_reduce(t, self._max())
            mine = t[self.rank * per:(self.rank + 1) * per].contiguous()
        local = torch.from_numpy(self.ops.count_raw(mine).astype(np.int64))
        if self.use_reduce_scatter:
            local = local.to(t.device)
        gathered = [torch.zeros_like(local) for _ in range(self.world)]
        self.dist.all_gather(gathered, local, group=self.group)
        return torch.cat([g.cpu() for g in gathered]).numpy()[:G].astype(np.uint64)
