"""Key-sharded sketch state across GPUs (one process per GPU).

The reference scales by running N processor processes on a Pulsar Shared
subscription (attendance_processor.py:30-34) against ONE Redis that
serialises every BF / PF op, so every process sees every key
(:127-129 writes it, :152 reads it).  Here every GPU holds:

  * a replica of the Bloom chain (read-only on the hot path; preload is
    replayed on every rank -- BF.MADD is deterministic);
  * the HLL keys it owns.

ONE ownership rule serves every multi-GPU path (``KeyMap``):

  owner(key)      = MurmurHash64A(key name, 0) mod world
  local slot      = the key's rank among the keys of its owner, in the order
                    of the job's key universe (every rank derives the same
                    table from the same names)

  * ingest routing (``route``) sends a swipe to owner(key) -- the hot path
    then has no exchange;
  * unpartitioned input (``SwipeExchange``) carries GLOBAL key indices into
    the universe and maps them through the same table on the device;
  * cross-shard queries (``ShardedSketch``) name keys, resolved to local
    slots through the client's key table, which ``KeyMap.bind`` fills with
    exactly the slots the other two paths write.

Queries that span shards use one RCCL collective on u8 register arrays with
MAX (HLL merge is an elementwise max, so the result is bit-identical to a
single-GPU run):

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
import math
from typing import Sequence

import numpy as np

from .encoding import encode
from .keyhash import murmur64a, murmur64a_many

HLL_REGISTERS = 16384
NO_SLOT = 0xFFFFFFFF  # a global key index outside the universe: K1 reports SKE_ERANGE


def owner(key, world: int) -> int:
    """Owner rank of one key name."""
    return murmur64a(encode(key), 0) % world


def route(keys: Sequence, world: int) -> np.ndarray:
    """Owner rank of every key (ingest routing of swipes): owner() per key."""
    return (murmur64a_many([encode(k) for k in keys], 0) % np.uint64(world)).astype(np.int32)


def balanced_owners(names: Sequence, world: int, weights=None, vbuckets: int | None = None) -> np.ndarray:
    """Mass-balanced ownership (an option beside north_star's hash rule):
    every key hashes to one of `vbuckets` virtual buckets (MurmurHash64A(key
    name, 0) mod V, default V = 256 x world), and the buckets go to ranks by
    greedy key mass -- heaviest bucket first, each to the rank with the least
    mass so far (ties: lower bucket, lower rank).  `weights`: each key's share
    of the stream (default 1 per key).  Deterministic, so every rank derives
    the same owners from the same names and weights.  Returns owner per key."""
    names = [encode(n) for n in names]
    V = int(vbuckets or 256 * world)
    vb = (murmur64a_many(names, 0) % np.uint64(V)).astype(np.int64) if names else np.zeros(0, np.int64)
    w = np.ones(len(names)) if weights is None else np.asarray(weights, np.float64)
    mass = np.bincount(vb, weights=w, minlength=V)
    order = np.lexsort((np.arange(V), -mass))
    load = np.zeros(world)
    assign = np.zeros(V, np.uint32)
    for b in order:
        r = int(np.argmin(load))  # the least-loaded rank (argmin: the lowest on ties)
        assign[b] = r
        load[r] += mass[b]
    return assign[vb]


class KeyMap:
    """The key namespace of a multi-GPU job.

    ``names[g]`` is global key ``g``; ``owner[g]`` = owner(names[g], world);
    ``local[g]`` = base(owner) + the position of g among the keys of that
    owner (increasing g).  ``base`` is an int or one int per rank (slots a
    rank keeps below the universe, e.g. another universe bound first).
    ``balance="mass"``: owners from balanced_owners(names, world, weights)
    instead of the hash rule (Zipf-skewed lecture popularity leaves the
    hash rule's heaviest rank ~10 % above the mean at 8 ranks, which bounds
    weak scaling; every path below reads ``owner`` from the map, so both
    rules serve ingest routing, the exchange and the planned queries alike;
    the name-based ShardedSketch queries take the map as ``keymap``)."""

    def __init__(self, names: Sequence, world: int, base=0, balance: str = "hash", weights=None,
                 vbuckets: int | None = None):
        self.names = [encode(n) for n in names]
        self.world = int(world)
        self.balance = balance
        if balance == "hash":
            self.owner = route(self.names, world).astype(np.uint32)
        elif balance == "mass":
            self.owner = balanced_owners(self.names, world, weights, vbuckets).astype(np.uint32)
        else:
            raise ValueError(f"unknown ownership rule {balance!r}")
        bases = [int(base)] * self.world if np.isscalar(base) else [int(b) for b in base]
        assert len(bases) == self.world
        self.base = bases
        self.local = np.empty(len(self.names), np.uint32)
        self._mine = []
        for r in range(self.world):
            idx = np.nonzero(self.owner == r)[0]
            self.local[idx] = bases[r] + np.arange(idx.size, dtype=np.uint32)
            self._mine.append(idx)
        self._dev = {}
        # one rank, no base: local slot = universe index
        self.identity = self.world == 1 and bases[0] == 0

    def __len__(self):
        return len(self.names)

    def owner_of(self, keys: Sequence) -> np.ndarray:
        """owner of each key name (names outside the universe: the hash rule)."""
        if not hasattr(self, "_index"):
            self._index = {n: g for g, n in enumerate(self.names)}
        out = np.empty(len(keys), np.int32)
        for i, k in enumerate(keys):
            g = self._index.get(encode(k))
            out[i] = self.owner[g] if g is not None else owner(k, self.world)
        return out

    def keys_of(self, rank: int) -> np.ndarray:
        """Global indices of the keys `rank` owns (increasing = local slot order)."""
        return self._mine[rank]

    def count(self, rank: int) -> int:
        return int(self._mine[rank].size)

    def slots_end(self, rank: int) -> int:
        """One past the last local slot of `rank` in this universe."""
        return self.base[rank] + self.count(rank)

    def bind(self, client, rank: int) -> None:
        """Name this rank's keys in the client's key table at their local
        slots (the slots K1 writes for them), so name-based queries --
        ShardedSketch, pfcount, hll_registers -- read what the hot path wrote."""
        for g in self._mine[rank]:
            client.keys.bind(self.names[g], int(self.local[g]))

    def tables(self, device):
        """(owner, local) as int32 torch tensors on `device` (cached)."""
        import torch
        key = str(device)
        if key not in self._dev:
            self._dev[key] = (torch.from_numpy(self.owner.view(np.int32)).to(device),
                              torch.from_numpy(self.local.view(np.int32)).to(device))
        return self._dev[key]

    def route_words(self) -> np.ndarray:
        """uint32 owner << 26 | local slot per key (ske_route_swipes_cap_async's
        key_route; local slots < 2^26 - 1, so no key packs to the no-owner word ~0)."""
        own = self.owner.astype(np.uint64)
        loc = self.local.astype(np.uint64)
        assert loc.size == 0 or int(loc.max()) < (1 << 26) - 1  # ~0 stays the no-owner word
        return ((own << np.uint64(26)) | loc).astype(np.uint32)

    def route_table(self, device):
        """route_words() as an int32 torch tensor on `device` (cached)."""
        import torch
        key = "route:" + str(device)
        if key not in self._dev:
            self._dev[key] = torch.from_numpy(self.route_words().view(np.int32)).to(device)
        return self._dev[key]


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
    """Name-based queries over keys spread by owner() across the ranks."""

    def __init__(self, client, rank: int, world: int, group=None, ops=None, keymap: KeyMap | None = None):
        import torch.distributed as dist
        self.dist = dist
        self.keymap = keymap  # a balanced ownership's map (None: the hash rule)
        self.client = client
        self.rank, self.world, self.group = rank, world, group
        self.ops = ops if ops is not None else LibsketchOps(client)
        backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
        self.use_reduce_scatter = backend == "nccl"
        self.solo = world == 1  # one shard (no process group needed): collectives are identities

    def _owned(self, keys: Sequence) -> np.ndarray:
        keys = list(keys)
        if not keys:
            return np.zeros(0, bool)
        if self.keymap is not None:
            return self.keymap.owner_of(keys) == self.rank
        return route(keys, self.world) == self.rank

    def owns(self, key) -> bool:
        return bool(self._owned([key])[0])

    def _max(self):
        return self.dist.ReduceOp.MAX

    def _all_reduce(self, t, op):
        """RCCL reduces device tensors in place; gloo (CPU tests, or ranks
        rehearsed on one GPU) gets a host copy of a device tensor."""
        if self.solo:
            return t
        if self.use_reduce_scatter or t.device.type == "cpu":
            self.dist.all_reduce(t, op=op, group=self.group)
            return t
        h = t.cpu()
        self.dist.all_reduce(h, op=op, group=self.group)
        t.copy_(h)
        return t

    def pfcount_union(self, keys: Sequence) -> int:
        keys = list(keys)
        m = self._owned(keys)
        t = self.ops.merge_groups([[k for k, o in zip(keys, m) if o]])
        self._all_reduce(t, self._max())
        return int(self.ops.count_raw(t)[0])

    def pfcount_each(self, keys: Sequence) -> np.ndarray:
        import torch
        keys = list(keys)
        idx = np.nonzero(self._owned(keys))[0]
        counts = np.zeros(len(keys), np.int64)
        if idx.size:
            counts[idx] = self.ops.count_each([keys[i] for i in idx]).astype(np.int64)
        if self.solo:
            return counts.astype(np.uint64)
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
        flat = [k for g in groups for k in g]
        m = iter(self._owned(flat).tolist())
        padded = [[k for k in g if next(m)] for g in groups] + [[]] * (per * self.world - G)
        t = self.ops.merge_groups(padded)
        if self.solo:
            return self.ops.count_raw(t)[:G].astype(np.uint64)
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


    # ---- planned queries: keys named by their global index in a KeyMap,
    # the name -> slot resolution done once (plan / plan_keys, kept on the
    # device), the query itself only device work and one collective
    # (C5's rankings, attendance_analysis.py:87-97 in PFCOUNT
    # form, and the campus PFMERGE).  Every library call is preceded by a
    # torch synchronisation: torch's stream and the context's stream are
    # different streams, and the plan's tensors, the output tensors and the
    # registers K1 wrote may still be in flight on either.
    def plan(self, keymap: KeyMap, groups: Sequence) -> dict:
        """This rank's part of every group of global key indices: the local
        slots of the keys it owns, groups padded to a multiple of world (the
        reduce_scatter split).  Slots and offsets are kept on the device too."""
        import torch
        G = len(groups)
        per = -(-G // self.world) if G else 0
        own, loc = keymap.owner, keymap.local
        parts, goffs = [], [0]
        for g in groups:
            g = np.asarray(g, np.int64)
            m = g[own[g] == self.rank] if g.size else g
            parts.append(loc[m].astype(np.uint32))
            goffs.append(goffs[-1] + int(m.size))
        goffs += [goffs[-1]] * (per * self.world - G)
        slots = np.concatenate(parts) if parts else np.zeros(0, np.uint32)
        dev = self.ops.device
        p = {"G": G, "per": per, "slots": slots, "goffs": np.asarray(goffs, np.uint32),
             "slots_dev": torch.from_numpy(slots.view(np.int32) if slots.size else np.zeros(1, np.int32)).to(dev),
             "goffs_dev": torch.from_numpy(np.asarray(goffs, np.uint32).view(np.int32)).to(dev)}
        self.torch_sync()
        return p

    def plan_keys(self, keymap: KeyMap, gidx) -> dict:
        """The plan of a key list (global indices) for pfcount_each_planned /
        pfmerge_planned: the positions of the keys this rank owns and their
        local slots, built once and kept on the device (the owner test and
        the slot lookup are not redone per query, and no slot list crosses
        the host link per query)."""
        import torch
        gidx = np.asarray(gidx, np.int64)
        pos = np.nonzero(keymap.owner[gidx] == self.rank)[0] if gidx.size else np.zeros(0, np.int64)
        slots = np.ascontiguousarray(keymap.local[gidx[pos]].astype(np.uint32))
        dev = self.ops.device
        ident = pos.size == gidx.size  # every key is this rank's (world 1): counts land in place
        kp = {"n": int(gidx.size), "mine": int(pos.size), "ident": ident,
              "slots_dev": torch.from_numpy(slots.view(np.int32) if slots.size else np.zeros(1, np.int32)).to(dev),
              "pos_dev": None if ident else torch.from_numpy(pos.astype(np.int64)).to(dev)}
        self.torch_sync()
        return kp

    def rollup_planned(self, plan: dict, device: bool = False):
        """rollup() of a plan: one union count per group.  One rank: the
        fused per-group K2 (merge + estimator, device arrays); N ranks: K3
        per group into a [groups, 16384] tensor, reduce_scatter MAX (RCCL),
        K2 estimator on this rank's share, all_gather of the counts.
        device=True: the counts stay on the device (an int64 tensor holding
        the u64 values), e.g. for rank_top_bottom_dev."""
        import torch
        G, per = plan["G"], plan["per"]
        dev = self.ops.device
        if self.solo:
            out = torch.empty(max(1, G), dtype=torch.int64, device=dev)
            if G:
                self.torch_sync()
                self.client.ctx.call("ske_hll_pfcount_groups", C.c_void_p(plan["slots_dev"].data_ptr()),
                                     C.c_void_p(plan["goffs_dev"].data_ptr()), G, C.c_void_p(out.data_ptr()), 1)
            return out[:G] if device else out[:G].cpu().numpy().astype(np.uint64)
        t = torch.zeros((per * self.world, HLL_REGISTERS), dtype=torch.uint8, device=dev)
        if per:
            self.torch_sync()
            self.client.ctx.call("ske_hll_merge_groups_dev", plan["slots"].ctypes.data_as(C.c_void_p),
                                 plan["goffs"].ctypes.data_as(C.c_void_p), per * self.world,
                                 C.c_void_p(t.data_ptr()))
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
        if device:
            return torch.cat([g.to(dev) for g in gathered])[:G]
        return torch.cat([g.cpu() for g in gathered]).numpy()[:G].astype(np.uint64)

    def pfcount_each_planned(self, kp, gidx=None):
        """PFCOUNT of every key of a plan_keys() plan (or of a KeyMap and
        global indices, planned on the spot), as a device int64 tensor
        holding the u64 counts: each rank counts its own keys (K2 per key,
        device slot list, the counts written in place at world 1 or
        scattered to their positions), then all_reduce SUM of the counts."""
        import torch
        if isinstance(kp, KeyMap):
            kp = self.plan_keys(kp, gidx)
        n, mine = kp["n"], kp["mine"]
        dev = self.ops.device
        if kp["ident"]:
            counts = out = torch.empty(max(1, n), dtype=torch.int64, device=dev)
        else:
            counts = torch.zeros(max(1, n), dtype=torch.int64, device=dev)
            out = torch.empty(max(1, mine), dtype=torch.int64, device=dev)
        if mine:
            self.torch_sync()
            self.client.ctx.call("ske_hll_pfcount_each", C.c_void_p(kp["slots_dev"].data_ptr()), mine,
                                 C.c_void_p(out.data_ptr()), 1)
            if not kp["ident"]:
                counts[kp["pos_dev"]] = out[:mine]
        if not self.solo:
            self._all_reduce_sum(counts)
        return counts[:n]

    def pfmerge_planned(self, kp, scratch_slot: int, gidx=None) -> tuple:
        """The campus PFMERGE of every key of a plan_keys() plan: each rank
        merges its own keys into `scratch_slot` (cleared first; the two-level
        K3 over the plan's device slot list, ske_hll_pfmerge_dev), the 16 KiB
        rows are max-reduced (all_reduce MAX) and counted.  Returns (PFCOUNT
        of the union, the union's registers as a uint8 tensor)."""
        import torch
        if isinstance(kp, KeyMap):
            kp = self.plan_keys(kp, gidx)
        ctx = self.client.ctx
        ctx.call("ske_hll_clear", int(scratch_slot))
        if kp["mine"]:
            self.torch_sync()
            ctx.call("ske_hll_pfmerge_dev", int(scratch_slot), C.c_void_p(kp["slots_dev"].data_ptr()), kp["mine"])
        p, nb = C.c_void_p(), C.c_uint64()
        ctx.call("ske_hll_slab", C.byref(p), C.byref(nb))
        row = torch.empty((1, HLL_REGISTERS), dtype=torch.uint8, device=self.ops.device)
        self.torch_sync()
        ctx.call("ske_memcpy", C.c_void_p(row.data_ptr()), C.c_void_p(p.value + int(scratch_slot) * HLL_REGISTERS),
                 HLL_REGISTERS, 3)
        self._all_reduce(row, self._max())
        return int(self.ops.count_raw(row)[0]), row

    def torch_sync(self):
        import torch
        if self.ops.device.type == "cuda":
            torch.cuda.synchronize(self.ops.device)

    def _all_reduce_sum(self, t):
        if self.use_reduce_scatter or t.device.type == "cpu":
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
            return t
        h = t.cpu()
        self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM, group=self.group)
        t.copy_(h)
        return t


class SwipeExchange:
    """Swipes that arrive NOT partitioned by key owner ("if
    input is not pre-partitioned, use one alltoallv per batch").

    Every rank holds an arbitrary slice of the stream: fixed-width ids and
    GLOBAL key indices into ``keymap``'s universe.  Global key ``g`` is owned
    by ``keymap.owner[g]`` as its local slot ``keymap.local[g]`` -- the rule
    ``route`` and ``ShardedSketch`` use.  One call:

      1. counting sort of the batch by owner (device: ``ske_route_swipes``
         through the key map's tables; CPU tensors: ``argsort``);
      2. ``all_to_all_single`` of the per-owner counts, then of the ids and
         of the local slots (RCCL over xGMI; variable splits = alltoallv);
      3. K1 on the received swipes (``k1(ids, local_slots) -> answers``);
      4. the answers back to their origin with the reverse splits, then
         un-permuted, so the caller gets BF.EXISTS per swipe in its own order.

    The registers end up exactly as if every swipe had been sent to its
    owner at ingest (PFADD is a per-register max).  A global index outside
    the universe travels to rank 0 with slot ``NO_SLOT``: its answer is
    still given, its PFADD dropped and reported as SKE_ERANGE by K1.  With
    ``gloo`` (CPU tests, or ranks rehearsed on one GPU) the collectives run
    on host copies.
    """

    def __init__(self, rank: int, world: int, k1, keymap: KeyMap, group=None, engine=None,
                 sink_slots=None, slack: float = 0.15, overlap: bool = True):
        import torch
        import torch.distributed as dist
        assert keymap.world == world, "the key map was built for another world size"
        self.torch, self.dist = torch, dist
        self.rank, self.world, self.k1, self.group = rank, world, k1, group
        self.keymap = keymap
        # with an engine, device batches are sorted / returned by the native
        # routing kernels (ske_route_swipes / ske_route_return_async,
        # sketch_route.hip); without one (CPU tensors) by torch ops
        self.engine = engine
        backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
        self.device_collectives = backend == "nccl"
        self.solo = world == 1  # one rank (no process group needed): the exchange is local
        # swipes_async: sink_slots[r] = a local slot rank r keeps for no key
        # (it absorbs the padding rows' PFADDs); slack = capacity over an
        # even share, adapted by settle() to the largest share it has seen
        self.sink = None if sink_slots is None else np.asarray(sink_slots, np.int64).astype(np.uint32)
        assert self.sink is None or self.sink.size == world
        self.slack = float(slack)
        self.pending = []
        self._free_pinned = []
        self.stats = {"batches": 0, "redone": 0, "max_share": 0.0}
        # swipes_async on a device with an engine: the pipelined form (routing
        # and the forward all_to_all of batch j+1 on a stream of their own
        # while batch j's K1 runs; see _swipes_async_pipelined)
        self.overlap = bool(overlap)
        self._pipe = None          # two parities of send / receive rows
        self._pipe_j = 0
        self._pipe_back = None     # the batch whose return half is not yet issued

    def capacity(self, n_max: int) -> int:
        """Rows per peer of the equal-split exchange for batches of at most
        n_max swipes (the same on every rank: a function of n_max, the world
        size and the slack every rank derives alike)."""
        if self.world == 1:
            return max(1, int(n_max))
        return min(int(n_max), math.ceil(int(n_max) * (1.0 + self.slack) / self.world)) + 256

    def owner_local(self, gkeys):
        """(owner, local slot) of global key indices (torch tensors)."""
        torch = self.torch
        own, loc = self.keymap.tables(gkeys.device)
        n = len(self.keymap)
        g = gkeys.to(torch.int64)
        inside = (g >= 0) & (g < n)
        gc = torch.where(inside, g, torch.zeros_like(g))
        dest = torch.where(inside, own[gc].to(torch.int64), torch.zeros_like(g))
        local = torch.where(inside, loc[gc], torch.full_like(loc[gc], -1))  # -1 = NO_SLOT as int32
        return dest, local

    def _a2a(self, out, inp, out_splits, in_splits):
        if self.solo:  # one rank (no process group): everything is local
            out.copy_(inp)
            return out
        if self.device_collectives or inp.device.type == "cpu":
            self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)
            return out
        o = out.cpu()
        self.dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
        out.copy_(o)
        return out

    def _on_stream(self, t):
        """libsketch follows torch's current stream, but a NULL handle (torch's
        default stream) means the library's own non-blocking stream, which
        does not order with torch's copies: on the default stream the
        exchange runs on a stream of its own, behind the caller's work, and
        the caller's stream waits for it at the end."""
        import contextlib
        torch = self.torch
        if not t.is_cuda or torch.cuda.current_stream(t.device).cuda_stream != 0:
            return contextlib.nullcontext(None)

        @contextlib.contextmanager
        def cm():
            caller = torch.cuda.current_stream(t.device)
            if not hasattr(self, "_own_stream"):
                self._own_stream = torch.cuda.Stream(t.device)
            s = self._own_stream
            s.wait_stream(caller)
            with torch.cuda.stream(s):
                yield caller
            caller.wait_stream(s)
        return cm()

    def swipes(self, ids, gkeys):
        """ids: uint8 [n, w] tensor, gkeys: integer [n] tensor of global key
        indices (same device).  Returns uint8 [n] answers in the input order."""
        with self._on_stream(ids) as caller:
            ans = self._swipes(ids, gkeys)
            if caller is not None:
                ans.record_stream(caller)
        return ans

    def _swipes(self, ids, gkeys):
        if self.engine is not None and ids.is_cuda:
            return self._swipes_native(ids, gkeys)
        torch = self.torch
        n, w = ids.shape
        dest, local = self.owner_local(gkeys)
        order = torch.argsort(dest, stable=True)
        send = torch.bincount(dest, minlength=self.world)
        recv = self._a2a(torch.empty_like(send), send, None, None)
        ins = send.cpu().tolist()
        outs = recv.cpu().tolist()
        m = int(sum(outs))
        # (16 zero bytes past the received ids: K1's short-id loads may read them)
        r_flat = torch.zeros(m * w + 16, dtype=torch.uint8, device=ids.device)
        r_ids = r_flat[:m * w].view(m, w)
        self._a2a(r_flat[:m * w], ids[order].reshape(-1), [c * w for c in outs], [c * w for c in ins])
        r_slots = torch.empty(m, dtype=torch.int32, device=ids.device)
        self._a2a(r_slots, local[order].to(torch.int32), outs, ins)
        r_ans = self.k1(r_ids, r_slots)
        back = torch.empty(n, dtype=torch.uint8, device=ids.device)
        self._a2a(back, r_ans.to(torch.uint8), ins, outs)
        ans = torch.empty_like(back)
        ans[order] = back
        return ans

    # ---- host-free form: equal splits of `cap` rows per peer
    def swipes_async(self, ids, gkeys, n_max: int | None = None, inputs_stable: bool = True):
        """``swipes`` with no host synchronisation (enqueue only on a device).

        Every peer pair exchanges exactly ``cap = capacity(n_max)`` rows
        (n_max: the largest batch any rank passes in this call; default this
        batch's size, so ranks must then pass equal sizes), so the splits are
        known without reading the routing counts: owner o's swipes fill rows
        [o*cap, o*cap + count_o), the rest are padding (zero ids into the
        owner's sink slot).  The answers tensor is returned at once and is
        final after ``settle()``, which every rank calls at the same point:
        a batch in which some owner got more than cap swipes on any rank is
        then run again through ``swipes`` (exact splits; PFADD is idempotent
        and its answers are rewritten).

        That re-run reads ``ids`` and ``gkeys`` again: they must hold the
        same swipes until ``settle()`` returns.  A caller that refills its
        input buffers sooner (a ring buffer) passes ``inputs_stable=False``,
        and the batch is kept as a device copy (one more read + write of
        its ids and keys) instead of by reference."""
        if not inputs_stable:
            ids, gkeys = ids.clone(), gkeys.clone()
        with self._on_stream(ids) as caller:
            ans = self._swipes_async(ids, gkeys, n_max)
            if caller is not None:
                ans.record_stream(caller)
        return ans

    def _swipes_async(self, ids, gkeys, n_max):
        torch = self.torch
        if self.sink is None:
            raise ValueError("swipes_async needs sink_slots (one spare local slot per rank)")
        n, w = ids.shape
        cap = self.capacity(n if n_max is None else n_max)
        assert n <= (n if n_max is None else n_max)
        dev = ids.device
        if self.solo and self.engine is not None and ids.is_cuda:
            return self._swipes_async_solo(ids, gkeys, n, w, cap)
        if self.overlap and self.engine is not None and ids.is_cuda:
            return self._swipes_async_pipelined(ids, gkeys, n, w, cap)
        if self.engine is not None and ids.is_cuda:
            send_ids, send_slots, pos, counts = self._route_cap_native(ids, gkeys, cap)
        else:
            send_ids, send_slots, pos, counts = self._route_cap_torch(ids, gkeys, cap)
        rows = self.world * cap
        # the capacity and slack these rows were sized with (settle() may
        # adapt the slack for the next batches)
        self.stats["cap_rows_per_peer"] = cap
        self.stats["slack_used"] = self.slack
        if self.world == 1:
            # one rank: the exchange is the identity, K1 reads the send rows
            # in place (their storage has the 16 readable bytes K1 wants)
            r_ids, r_slots = send_ids, send_slots
        else:
            r_flat = torch.zeros(rows * w + 16, dtype=torch.uint8, device=dev)
            self._a2a(r_flat[:rows * w], send_ids.reshape(-1), None, None)
            r_ids = r_flat[:rows * w].view(rows, w)
            r_slots = torch.empty(rows, dtype=torch.int32, device=dev)
            self._a2a(r_slots, send_slots, None, None)
        r_ans = self.k1(r_ids, r_slots).to(torch.uint8)
        if self.world == 1:
            back = r_ans
        else:
            back = torch.empty(rows, dtype=torch.uint8, device=dev)
            self._a2a(back, r_ans, None, None)
        ans = self._gather(back, pos, n)
        if counts.is_cuda:
            # pinned landing rows for the counts, reused once settled
            host = self._free_pinned.pop() if self._free_pinned else \
                torch.empty(self.world, dtype=torch.int32, pin_memory=True)
            host.copy_(counts, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = counts.to(torch.int32), None
        self.pending.append({"ids": ids, "gkeys": gkeys, "ans": ans, "counts": host, "ev": ev, "cap": cap,
                             "n": n})
        return ans

    def settle(self) -> int:
        """Finish every swipes_async batch since the last settle (collective:
        every rank calls it at the same point).  Returns the batches re-run
        because some owner overflowed its capacity on some rank; adapts the
        slack to the largest owner share seen (the same on every rank)."""
        torch = self.torch
        self.flush()
        pend, self.pending = self.pending, []
        if not pend:
            return 0
        flags, share = [], 0.0
        for p in pend:
            if p["ev"] is not None:
                p["ev"].synchronize()
            c = p["counts"].numpy().astype(np.int64)
            if p["ev"] is not None:
                self._free_pinned.append(p["counts"])
            flags.append(int(c.max(initial=0) > p["cap"]))
            if p["n"]:
                share = max(share, float(c.max(initial=0)) * self.world / p["n"])
        v = torch.tensor(flags + [int(share * 1e6)], dtype=torch.int64)
        if not self.solo:
            if self.device_collectives:
                v = v.to(pend[0]["ans"].device)
            self.dist.all_reduce(v, op=self.dist.ReduceOp.MAX, group=self.group)
            v = v.cpu()
        v = v.tolist()
        redo = 0
        for p, f in zip(pend, v[:-1]):
            if f:
                p["ans"].copy_(self.swipes(p["ids"], p["gkeys"]))
                redo += 1
        gshare = v[-1] / 1e6
        self.stats["batches"] += len(pend)
        self.stats["redone"] += redo
        self.stats["max_share"] = max(self.stats["max_share"], gshare)
        if gshare > 0:
            self.slack = max(0.02, gshare - 1.0 + 0.03)
        return redo

    # ---- one rank: the exchange is the identity
    def _swipes_async_solo(self, ids, gkeys, n, w, cap):
        """World 1 (no process group): every key is this rank's, so nothing
        is sorted, sent or gathered back -- the keys are mapped to local
        slots (ske_route_slots_async, 8 B per swipe) and K1 reads the ids in
        place, answering in input order.  (K1 may read up to 16 bytes past
        the last id: ids whose storage ends at the last id are copied into a
        padded buffer first.)"""
        torch = self.torch
        dev = ids.device
        ids = ids.contiguous()
        end = ids.storage_offset() * ids.element_size() + n * w
        if ids.untyped_storage().nbytes() - end < 16:
            pad = torch.empty(n * w + 16, dtype=torch.uint8, device=dev)
            pad[:n * w].view(n, w).copy_(ids)
            ids = pad[:n * w].view(n, w)
        g32 = gkeys.to(torch.int32).contiguous()
        # a one-rank key map is the identity (local slot = universe index):
        # no table, the kernel only checks the range
        kroute = None if getattr(self.keymap, "identity", False) else self.keymap.route_table(dev)
        slots = torch.empty(max(1, n), dtype=torch.int32, device=dev)
        eng = self.engine
        prev = eng.get_stream()
        try:
            eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            eng.ctx.call("ske_route_slots_async", C.c_void_p(g32.data_ptr()), n,
                         C.c_void_p(None if kroute is None else kroute.data_ptr()),
                         len(self.keymap), self.world, C.c_void_p(slots.data_ptr()))
        finally:
            eng.set_stream(prev)
        self.stats["cap_rows_per_peer"] = cap
        self.stats["slack_used"] = self.slack
        ans = self.k1(ids, slots[:n]).to(torch.uint8)
        self.pending.append({"ids": ids, "gkeys": gkeys, "ans": ans, "counts": torch.tensor([n], dtype=torch.int32),
                             "ev": None, "cap": cap, "n": n})
        return ans

    # ---- the pipelined form of swipes_async
    #
    # Three streams besides the caller's: R (routing, the forward
    # all_to_all_single of ids and slots), K (K1), B (the answers'
    # all_to_all_single back, the gather into input order).  Batch j:
    #
    #   caller: event "inputs ready"        R: wait it; wait rows[j % 2] free;
    #   route j; counts -> pinned host; forward a2a j     K: wait R; K1 j
    #   (batch j-1's return half is issued here, AFTER batch j's forward
    #   all_to_all: collectives of one process group run in issue order, so a
    #   return of j-1 issued first would hold j's forward behind K1 j-1)
    #   B (issued with batch j+1 or by flush): wait K1 j; a2a back; gather;
    #   event "rows[j % 2] free"
    #
    # so batch j+1's routing and forward exchange run while batch j's K1 does,
    # and two parities of send / receive rows keep them apart.  The answers
    # are final after settle() (as in the one-stream form); flush() issues
    # the last return half and makes the caller's stream wait for all three
    # streams without a host synchronisation.
    def _pipe_rows(self, dev, rows, w, n):
        """the two parities of rows for `rows` send rows of w bytes and a
        batch of n swipes (pos holds one entry per swipe: n exceeds rows when
        a capacity below the owners' shares is asked for)"""
        torch = self.torch
        if self._pipe is not None and self._pipe_key == (rows, w, dev) and self._pipe[0]["pos"].numel() >= n:
            return self._pipe
        self.flush()
        if self._pipe is not None:
            torch.cuda.current_stream(dev).synchronize()  # (old rows: nothing may still use them)
        solo = self.world == 1

        def parity():
            return {"send_ids": torch.empty(rows * w + 16, dtype=torch.uint8, device=dev),
                    "send_slots": torch.empty(rows, dtype=torch.int32, device=dev),
                    "pos": torch.empty(max(1, rows, n), dtype=torch.int32, device=dev),
                    "counts": torch.empty(self.world, dtype=torch.int32, device=dev),
                    "r_flat": None if solo else torch.zeros(rows * w + 16, dtype=torch.uint8, device=dev),
                    "r_slots": None if solo else torch.empty(rows, dtype=torch.int32, device=dev),
                    "back": None if solo else torch.empty(rows, dtype=torch.uint8, device=dev),
                    "free": None}
        if not hasattr(self, "_pipe_streams") or self._pipe_streams[0].device != dev:
            # (the return half on K1's stream, or the routing stream at high
            # priority, measured no different at N = 1: profiles/r05_exchange_overlap.txt)
            self._pipe_streams = tuple(torch.cuda.Stream(dev) for _ in range(3))
        self._pipe = [parity(), parity()]
        self._pipe_key = (rows, w, dev)
        return self._pipe

    def _swipes_async_pipelined(self, ids, gkeys, n, w, cap):
        torch = self.torch
        dev = ids.device
        rows = self.world * cap
        pipe = self._pipe_rows(dev, rows, w, n)
        sr, sk, sb = self._pipe_streams
        caller = torch.cuda.current_stream(dev)
        ready = torch.cuda.Event()
        ready.record(caller)
        B = pipe[self._pipe_j % 2]
        self._pipe_j += 1
        self.stats["cap_rows_per_peer"] = cap
        self.stats["slack_used"] = self.slack
        sr.wait_event(ready)
        if B["free"] is not None:
            sr.wait_event(B["free"])
        with torch.cuda.stream(sr):
            send_ids, send_slots, pos, counts = self._route_cap_native(ids, gkeys, cap, bufs=B)
            host = self._free_pinned.pop() if self._free_pinned else \
                torch.empty(self.world, dtype=torch.int32, pin_memory=True)
            host.copy_(counts, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(sr)
            if self.world == 1:
                r_ids, r_slots = send_ids, send_slots
            else:
                self._a2a(B["r_flat"][:rows * w], send_ids.reshape(-1), None, None)
                self._a2a(B["r_slots"], send_slots, None, None)
                r_ids, r_slots = B["r_flat"][:rows * w].view(rows, w), B["r_slots"]
            fwd = torch.cuda.Event()
            fwd.record(sr)
        self._issue_back()  # batch j-1's return half, behind batch j's forward exchange
        sk.wait_event(fwd)
        with torch.cuda.stream(sk):
            r_ans = self.k1(r_ids, r_slots)
            done = torch.cuda.Event()
            done.record(sk)
        ans = torch.empty(n, dtype=torch.uint8, device=dev)
        self._pipe_back = {"B": B, "r_ans": r_ans, "done": done, "n": n, "ans": ans, "rows": rows}
        self.pending.append({"ids": ids, "gkeys": gkeys, "ans": ans, "counts": host, "ev": ev, "cap": cap, "n": n})
        return ans

    def _issue_back(self):
        p, self._pipe_back = self._pipe_back, None
        if p is None:
            return
        torch = self.torch
        sr, sk, sb = self._pipe_streams
        B = p["B"]
        sb.wait_event(p["done"])
        with torch.cuda.stream(sb):
            if self.world == 1:
                back = p["r_ans"]
            else:
                back = B["back"]
                self._a2a(back, p["r_ans"], None, None)
            self._gather(back, B["pos"], p["n"], ans=p["ans"])
            free = torch.cuda.Event()
            free.record(sb)
        B["free"] = free
        # (the allocator may hand these out again only after stream B's use)
        p["r_ans"].record_stream(sb)
        p["ans"].record_stream(sb)

    def flush(self):
        """Issue the pipelined form's last return half and make the caller's
        stream wait for the exchange's streams (no host synchronisation):
        after it, work on the caller's stream sees every answer."""
        if self._pipe is None:
            return
        self._issue_back()
        torch = self.torch
        caller = torch.cuda.current_stream(self._pipe_key[2])
        for s_ in self._pipe_streams:
            caller.wait_stream(s_)

    def _route_cap_torch(self, ids, gkeys, cap):
        torch = self.torch
        n, w = ids.shape
        dest, local = self.owner_local(gkeys)
        order = torch.argsort(dest, stable=True)
        counts = torch.bincount(dest, minlength=self.world)
        starts = torch.cumsum(counts, 0) - counts
        ds = dest[order]
        r = torch.arange(n, device=ids.device) - starts[ds]
        keep = r < cap
        row = ds * cap + torch.where(keep, r, r % cap)
        rows = self.world * cap
        send_ids = torch.zeros(rows * w + 16, dtype=torch.uint8, device=ids.device)[:rows * w].view(rows, w)
        sink = torch.from_numpy(self.sink.astype(np.int64)).to(torch.int32).to(ids.device)
        send_slots = sink[torch.arange(rows, device=ids.device) // cap]
        send_ids[row[keep]] = ids[order][keep]
        send_slots[row[keep]] = local[order][keep].to(torch.int32)
        pos = torch.empty(n, dtype=torch.int64, device=ids.device)
        pos[order] = row
        return send_ids, send_slots, pos, counts

    def _route_cap_native(self, ids, gkeys, cap, bufs=None):
        torch = self.torch
        n, w = ids.shape
        dev = ids.device
        ids = ids.contiguous()
        g32 = gkeys.to(torch.int32).contiguous()
        kroute = self.keymap.route_table(dev)
        rows = self.world * cap
        if bufs is None:
            send_ids = torch.empty(rows * w + 16, dtype=torch.uint8, device=dev)  # + K1's readable tail
            send_slots = torch.empty(rows, dtype=torch.int32, device=dev)
            pos = torch.empty(max(1, n), dtype=torch.int32, device=dev)
            counts = torch.empty(self.world, dtype=torch.int32, device=dev)
        else:
            send_ids, send_slots, pos, counts = bufs["send_ids"], bufs["send_slots"], bufs["pos"], bufs["counts"]
            # (the kernels write n positions, rows ids and slots, world counts)
            if (send_ids.numel() < rows * w + 16 or send_slots.numel() < rows or pos.numel() < max(1, n)
                    or counts.numel() < self.world):
                raise ValueError("SwipeExchange: routing rows smaller than the batch")
        if not hasattr(self, "_sink_dev"):
            self._sink_dev = torch.from_numpy(self.sink.view(np.int32)).to(dev)
        eng = self.engine
        prev = eng.get_stream()
        try:
            eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            eng.ctx.call("ske_route_swipes_cap_async", C.c_void_p(ids.data_ptr()), w, C.c_void_p(g32.data_ptr()), n,
                         self.world, C.c_void_p(kroute.data_ptr()), len(self.keymap),
                         cap, C.c_void_p(self._sink_dev.data_ptr()), C.c_void_p(send_ids.data_ptr()),
                         C.c_void_p(send_slots.data_ptr()), C.c_void_p(pos.data_ptr()),
                         C.c_void_p(counts.data_ptr()))
        finally:
            eng.set_stream(prev)
        return send_ids[:rows * w].view(rows, w), send_slots, pos, counts

    def _gather(self, back, pos, n, ans=None):
        """answers of the send rows back into input order"""
        torch = self.torch
        if self.engine is not None and back.is_cuda:
            if ans is None:
                ans = torch.empty(n, dtype=torch.uint8, device=back.device)
            eng = self.engine
            prev = eng.get_stream()
            try:
                eng.set_stream(torch.cuda.current_stream(back.device).cuda_stream)
                eng.ctx.call("ske_route_return_async", C.c_void_p(back.data_ptr()), C.c_void_p(pos.data_ptr()), n,
                             C.c_void_p(ans.data_ptr()))
            finally:
                eng.set_stream(prev)
            return ans
        return back[pos[:n].to(torch.int64)]

    def _swipes_native(self, ids, gkeys):
        torch = self.torch
        n, w = ids.shape
        dev = ids.device
        ids = ids.contiguous()
        g32 = gkeys.to(torch.int32).contiguous()
        own, loc = self.keymap.tables(dev)
        sids = torch.empty(n * w, dtype=torch.uint8, device=dev)
        sslot = torch.empty(n, dtype=torch.int32, device=dev)
        pos = torch.empty(n, dtype=torch.int32, device=dev)
        counts = np.zeros(self.world, np.uint64)
        eng = self.engine
        prev = eng.get_stream()
        try:
            eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            eng.ctx.call("ske_route_swipes", C.c_void_p(ids.data_ptr()), w, C.c_void_p(g32.data_ptr()), n,
                         self.world, C.c_void_p(own.data_ptr()), C.c_void_p(loc.data_ptr()), len(self.keymap),
                         C.c_void_p(sids.data_ptr()), C.c_void_p(sslot.data_ptr()),
                         C.c_void_p(pos.data_ptr()), counts.ctypes.data_as(C.c_void_p))
            send = torch.from_numpy(counts.astype(np.int64))
            if self.device_collectives:
                send = send.to(dev)
            recv = self._a2a(torch.empty_like(send), send, None, None)
            ins = [int(c) for c in counts]
            outs = recv.cpu().tolist()
            m = int(sum(outs))
            r_flat = torch.zeros(m * w + 16, dtype=torch.uint8, device=dev)
            r_ids = r_flat[:m * w].view(m, w)
            self._a2a(r_flat[:m * w], sids, [c * w for c in outs], [c * w for c in ins])
            r_slots = torch.empty(m, dtype=torch.int32, device=dev)
            self._a2a(r_slots, sslot, outs, ins)
            r_ans = self.k1(r_ids, r_slots)
            back = torch.empty(n, dtype=torch.uint8, device=dev)
            self._a2a(back, r_ans.to(torch.uint8), ins, outs)
            ans = torch.empty(n, dtype=torch.uint8, device=dev)
            eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            eng.ctx.call("ske_route_return_async", C.c_void_p(back.data_ptr()), C.c_void_p(pos.data_ptr()), n,
                         C.c_void_p(ans.data_ptr()))
        finally:
            eng.set_stream(prev)
        return ans


class _Ptr:
    def __init__(self, p: int):
        self.ptr = p


class _FixedBatch:
    """A fixed-width batch over torch tensors, as the engine's K1 calls read it."""

    def __init__(self, ids, slots):
        self.n, self.width = int(ids.shape[0]), int(ids.shape[1])
        self.bytes, self.slot = _Ptr(ids.data_ptr()), _Ptr(slots.data_ptr())


def engine_k1(engine, fid: int = 0):
    """``SwipeExchange``'s K1 on this rank's GPU: the received fixed-width ids
    and local slots (device tensors; the ids' storage has 16 readable bytes
    past the last id) through ske_swipes_fixed_async on torch's current
    stream (the engine's stream is restored afterwards)."""
    import torch

    def k1(ids, slots):
        out = torch.empty(ids.shape[0], dtype=torch.uint8, device=ids.device)
        if ids.shape[0]:
            prev = engine.get_stream()
            try:
                engine.set_stream(torch.cuda.current_stream(ids.device).cuda_stream)
                engine.swipes_fixed_async(fid, _FixedBatch(ids, slots.contiguous()), _Ptr(out.data_ptr()))
            finally:
                engine.set_stream(prev)
        return out

    return k1
