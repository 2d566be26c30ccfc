"""Benchmark of the fused validate-and-count hot path (K1: BF.EXISTS +
valid-gated PFADD) -- BASELINE.json's metric on its north-star configuration.

Default workload: C3 (configs[2], the configuration BASELINE.md quotes the
1/2/4/8-GPU curve on), this rank's shard of it: the replicated 10M-student
Bloom filter (RESERVE 0.001 / 1e7: 19.8 MB, k = 11) preloaded by BF.MADD, a
Zipf(1.1)-over-lectures x uniform-over-days stream of 8-digit ids with 10 %
invalid swipes, and this rank's HLL keys (100k at N = 1, 12.5k per rank at
N = 8; synthetic.shard).  One step = one K1 call over one resident batch of
16M swipes (answers written, PFADD of the valid ones): the partitioned K1,
three kernels (sketch_part.hip: hash + probe records, LDS-slice probes,
answers + register max).  `--config c2` runs C2 (1M swipes, the LDS K1).

Inputs are generated on the GPU and resident in HBM before timing; every
step consumes a distinct batch of the stream.  Timing: W untimed warm-up
steps, then K steps bracketed by barrier + synchronize; value = swipes of all
ranks / the slowest rank's wall time.  With the library's pass timing on,
every K1 kernel of the timed steps is bracketed by a HIP event pair on the
stream it runs on (ske_pass_times): the roofline is priced on the kernel that
takes the most time, from those live durations.

N>1: one process per GPU (torch.distributed.run), RCCL ("nccl") process
group; every rank runs its own stream over its own key shard with the Bloom
replicated (no data-path collective; weak scaling).  After timing, every rank
checks a verification batch against the CPU oracle and the cross-shard
queries (all_reduce MAX union, reduce_scatter MAX rollup) against the same
collectives over the oracle's registers; the line carries the outcome under
"check".

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# tools/randbench.hip on MI355X (profiles/r02_randbench.json): one random
# 4-byte read per lane over a 1.6 GB table -- 55 G sectors/s; the register
# update of pass C is priced against it as well as against the HBM peak
RANDOM_SECTOR_GPS = 55.3
# tools/casbench.hip (profiles/r02_casbench.json): pass C's own operation in
# isolation -- load a random word of a 1.6 GB table, raise one byte by a CAS on
# it -- 21.1 G ops/s at 7.3 M ops (device-scope atomics execute memory-side:
# TCC_EA0_ATOMIC); pass C's register CASes are priced against it
RANDOM_CAS_GPS = 21.1
MALL_BYTES = 256 << 20  # Infinity Cache: a slab this small stays on chip
METRIC = "swipes/sec (fused BF.EXISTS+PFADD) at 1/2/4/8 GPUs; % of HBM peak"
PASS_NAMES = ["k1", "k_part_a", "k_part_b", "k_part_c"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--batch", type=int, default=0, help="swipes per step (default: config)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--tile", type=int, default=0, help="K1 swipes per thread in flight (1,2,4,8)")
    ap.add_argument("--variant", type=int, default=-1,
                    help="-1 auto, 0 global Bloom, 1 LDS Bloom, 2 XCD-partitioned, 3 partitioned")
    ap.add_argument("--max-batches", type=int, default=64)
    ap.add_argument("--ablate", type=int, default=0, help="diagnostic: K1 parts removed (bits)")
    ap.add_argument("--part-sub", type=int, default=0,
                    help="partitioned K1: swipes per sub-batch of its three passes (0 = default)")
    ap.add_argument("--hll-mode", type=int, default=-1,
                    help="partitioned K1 PFADD: 0 = CAS on the slab, 1 = owned register lines "
                         "(-1: library default)")
    ap.add_argument("--exchange", type=int, default=0,
                    help="1 = unpartitioned input: every rank's batches span ALL keys and a step "
                         "routes them to the key owners with all_to_all_single "
                         "(distributed.SwipeExchange), runs K1 there and returns the answers")
    ap.add_argument("--pa-tile", type=int, default=-1,
                    help="partitioned K1 tile: 10 = 1024 swipes, 11 = 2048 (one-link k = 11 "
                         "chains; -1: library default)")
    ap.add_argument("--pa-precheck", type=int, default=-1,
                    help="partitioned K1: 1 = pass A pre-checks the HLL registers (pass C only "
                         "raises), 0 = pass C loads them (-1: library default)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="library option (ske_set_option), e.g. part_overlap=2; repeatable")
    ap.add_argument("--pb-pairs", type=int, default=-1,
                    help="partitioned K1 pass B: 1 = slice pairs (128 KiB images), 0 = single "
                         "slices (-1: library default)")
    ap.add_argument("--persistent", type=int, default=-1,
                    help="1 = the K timed steps as ONE ske_swipes_many_async call (for the "
                         "partitioned K1 with the part_overlap option: each step's pass C on a side "
                         "stream beside the next step's pass B); for the LDS K1 one persistent "
                         "LDS K1 launch over the K batches; default for the LDS K1); 0 = a K1 "
                         "launch per step")
    ap.add_argument("--streams", type=int, default=0,
                    help="HIP streams / graph branches the steps alternate over (0: 16 for the "
                         "LDS K1, 1 otherwise)")
    ap.add_argument("--k1-grid", type=int, default=-1, help="blocks of the short-id LDS K1")
    ap.add_argument("--graph", type=int, default=-1,
                    help="1 = record the K timed steps into a HIP graph and replay it (default for "
                         "the LDS K1); 0 = launch them from the host (default otherwise)")
    ap.add_argument("--pass-timing", type=int, default=1,
                    help="1 = HIP events around every K1 kernel of the timed steps (host launches)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N>1 (nccl = RCCL over xGMI; gloo only to rehearse "
                         "several ranks on a one-GPU box)")
    ap.add_argument("--layout", default="offsets", choices=["offsets", "fixed"],
                    help="id batch layout: bytes + u32 offsets, or fixed-width ids")
    return ap.parse_args()


def cpu_threads():
    """Host threads for the all-cores CPU baseline: OMP_NUM_THREADS when set
    (the GPU box sets it to its CPU share, 16), else this process's affinity."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    n = int(env) if env.isdigit() and int(env) > 0 else len(os.sched_getaffinity(0))
    return max(1, min(n, 64))


def chain_geometry(engine, fid=0):
    """(bits, k) of every link of the chain (BF.DEBUG)."""
    from rtsas_amd._lib import BfInfo, BfLink
    info = BfInfo()
    engine.ctx.call("ske_bf_info", fid, C.byref(info))
    out = []
    for i in range(info.nfilters):
        li = BfLink()
        engine.ctx.call("ske_bf_link_info", fid, i, C.byref(li))
        out.append((int(li.bits), int(li.hashes)))
    return out


def oracle_chain(engine, orc, w, p):
    """The Bloom chain as the oracle builds it from the same preload (RedisBloom
    SBChain_Add restated, oracle/sketch_oracle.c) -- test infrastructure."""
    mb = engine.members_batch(p, 0, w.n_members)
    buf, offs, _ = mb.to_host()
    mb.free()
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    chain.madd_packed(buf, offs)
    return chain


def cpu_baseline(orc, chain, w, b0, seconds):
    """The processor loop attendance_processor.py:100-137 (BF.EXISTS, then
    PFADD when valid) on the host, over a bounded sample of the first batch:
      - the C oracle on all host threads (orc_process_swipes_mt; the value),
        and on one thread;
      - the reference's per-event Python loop (json.loads, fromisoformat,
        BF.EXISTS, PFADD per message) over the oracle, one core (§8d item 1)."""
    import numpy as np
    from datetime import datetime
    from rtsas_amd import synthetic
    buf, offs, slot = b0.to_host()
    n = min(len(offs) - 1, 1 << 20)
    offs = np.ascontiguousarray(offs[:n + 1])
    slot = np.ascontiguousarray(slot[:n].astype(np.uint32))
    regs = np.zeros((int(slot.max()) + 1, 16384), np.uint8)

    def run(threads, budget):
        passes, t0 = 0, time.perf_counter()
        while True:
            orc.process_swipes(chain, regs, slot, buf, offs, threads=threads)
            passes += 1
            if time.perf_counter() - t0 >= budget:
                return passes, time.perf_counter() - t0

    nt = cpu_threads()
    pm, dtm = run(nt, seconds * 0.45)
    p1, dt1 = run(1, seconds * 0.3)
    # per-event loop over JSON payloads of the generator's schema
    # (data_generator.py:112-118) carrying the same swipes
    m = 100_000
    msgs = []
    for i in range(m):
        sid = bytes(buf[offs[i]:offs[i + 1]]).decode()
        _, _, lecture, day = synthetic.key_name(w, int(slot[i])).split(":")
        msgs.append('{"student_id": %s, "timestamp": "%sT09:00:00", "lecture_id": "%s", '
                    '"is_valid": true, "event_type": "entry"}' % (sid, day, lecture))
    hlls = {}
    t0 = time.perf_counter()
    for msg in msgs:
        data = json.loads(msg)
        sid = str(data["student_id"]).encode()
        ts = datetime.fromisoformat(data["timestamp"])
        if chain.exists(sid):
            hlls.setdefault(f"hll:unique:{data['lecture_id']}:{ts.date().isoformat()}",
                            orc.HLL()).add(sid)
    dte = time.perf_counter() - t0
    return {"value": n * pm / dtm, "unit": "swipes/s", "cores": nt, "kind": "port",
            "sample": f"{pm} passes over the first {n} swipes of batch 0 (C oracle of RedisBloom + "
                      f"Redis HLL, orc_process_swipes_mt on {nt} threads, {dtm:.1f}s)",
            "single_thread": {"value": n * p1 / dt1, "cores": 1,
                              "sample": f"{p1} passes, orc_process_swipes, {dt1:.1f}s"},
            "per_event_python": {"value": m / dte, "cores": 1,
                                 "sample": f"{m} JSON messages: json.loads + fromisoformat + "
                                           "oracle BF.EXISTS / PFADD per event "
                                           "(attendance_processor.py:100-137 without transport)"}}


def verify(engine, orc, chain, w, rank, world, dist, dev):
    """A verification batch through K1 into 64 spare slots of this rank,
    compared with the oracle (answers + registers), then the cross-shard
    queries: union PFCOUNT of the 64 keys of every rank (all_reduce MAX) and
    the 64 per-key unions across ranks (reduce_scatter MAX), each against the
    same collective over the oracle's registers."""
    import numpy as np
    import torch
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer
    nk, base = 64, w.n_keys
    wv = synthetic.Workload(**{**w.__dict__, "n_keys": nk, "zipf_lectures": 0, "zipf_days": 0})
    pv = engine.gen_params(wv, seed=w.seed + 7919 * (rank + 1), slot_base=base)
    n = 1 << 19
    b = engine.swipe_batch(pv, 0, n)
    out = DeviceBuffer(engine.ctx, n)
    engine.swipes(0, b, out)
    buf, offs, slot = b.to_host()
    regs = np.zeros((nk, 16384), np.uint8)
    want, _, _ = orc.process_swipes(chain, regs, (slot - base).astype(np.uint32), buf, offs)
    ok_local = bool(np.array_equal(out.to_host(np.uint8, n), want)) and \
        bool(np.array_equal(engine.registers_all(base + nk)[base:], regs))
    b.free()
    out.free()
    slots = np.arange(base, base + nk, dtype=np.uint32)
    # union of the 64 keys of every rank: device merge -> all_reduce MAX -> K2
    t = torch.zeros((1, 16384), dtype=torch.uint8, device=dev)
    go = np.array([0, nk], np.uint32)
    torch.cuda.synchronize()
    engine.ctx.call("ske_hll_merge_groups_dev", slots.ctypes.data_as(C.c_void_p),
                    go.ctypes.data_as(C.c_void_p), 1, C.c_void_p(t.data_ptr()))
    o = torch.from_numpy(regs.max(axis=0, keepdims=True)).to(dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(o, op=dist.ReduceOp.MAX)
    torch.cuda.synchronize()
    union = np.zeros(1, np.uint64)
    engine.ctx.call("ske_hll_count_raw_dev", C.c_void_p(t.data_ptr()), 1,
                    union.ctypes.data_as(C.c_void_p))
    ok_union = bool(torch.equal(t, o)) and int(union[0]) == orc.hll_count_regs(o.cpu().numpy()[0])
    # per-key unions across ranks: reduce_scatter MAX, each rank owns 64/world keys
    per = -(-nk // world)
    tk = torch.zeros((per * world, 16384), dtype=torch.uint8, device=dev)
    gk = np.arange(nk + 1, dtype=np.uint32)
    engine.ctx.call("ske_hll_merge_groups_dev", slots.ctypes.data_as(C.c_void_p),
                    gk.ctypes.data_as(C.c_void_p), nk, C.c_void_p(tk.data_ptr()))
    tk_o = torch.zeros_like(tk)
    tk_o[:nk] = torch.from_numpy(regs).to(dev)
    mine = torch.empty((per, 16384), dtype=torch.uint8, device=dev)
    mine_o = torch.empty_like(mine)
    if world > 1:
        dist.reduce_scatter_tensor(mine, tk, op=dist.ReduceOp.MAX)
        dist.reduce_scatter_tensor(mine_o, tk_o, op=dist.ReduceOp.MAX)
    else:
        mine.copy_(tk)
        mine_o.copy_(tk_o)
    torch.cuda.synchronize()
    ok_rollup = bool(torch.equal(mine, mine_o))
    ok = torch.tensor([int(ok_local and ok_union and ok_rollup)], device=dev)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return {"ok": bool(ok.item()), "swipes_per_rank": n, "keys_per_rank": nk,
            "local_answers_and_registers": ok_local, "union_all_reduce_max": ok_union,
            "rollup_reduce_scatter_max": ok_rollup, "union_pfcount": int(union[0]),
            "backend": dist.get_backend() if world > 1 else "none"}


def pass_bytes(n, nvalid, probes, width, fixed, geometry, lds_k1=False, slab_bytes=0, cus=256):
    """Algorithmic bytes per launch of each K1 kernel: streams
    at their size, every random access at one 64-B HBM sector.  The LDS K1
    (lds_k1) reads the filter once per block (staged into LDS, probes cost no
    HBM) and its register words only when the slab does not fit on chip."""
    s_off = 0 if fixed else 4
    ksum = sum(k for _, k in geometry)
    nslices = sum(-(-bits // (1 << 19)) for bits, _ in geometry)
    filter_bytes = sum(bits // 8 for bits, _ in geometry)
    rec = 4 * ksum * n
    ntiles = -(-n // 1024)
    return {
        # one kernel: ids + offsets + slot + answer streamed, one sector per
        # RedisBloom probe, one sector read + one written per valid swipe
        "k1": (n * (width + s_off + 4 + 1)
               + (128 * nvalid if slab_bytes > MALL_BYTES else 0)) if lds_k1 else
              n * (width + s_off + 4 + 1) + 64 * probes + 128 * nvalid,
        # the LDS K1 stages the filter into every block's LDS once per launch
        "k1_stage": filter_bytes * cus if lds_k1 else 0,
        # ids + offsets in; probe records, run table, HLL word, fail byte out
        "k_part_a": n * (width + s_off) + rec + 4 * (nslices + 1) * ntiles + 4 * n + n * len(geometry),
        # probe records + their run boundaries in, the filter staged once
        "k_part_b": rec + 8 * nslices * ntiles + filter_bytes,
        # fail byte, HLL word, slot in, answer out; per valid swipe its register's
        # sector read + written (SURVEY §8d's 128·v, as the one-kernel K1 above)
        "k_part_c": n * (len(geometry) + 4 + 4 + 1) + 128 * nvalid,
    }


def main():
    args = parse()
    import numpy as np  # noqa: F401
    import torch
    import torch.distributed as dist

    import __graft_entry__ as ge
    ge.load_package()
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer, SketchEngine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one GPU per rank; the modulo only matters for a rehearsal of several
    # ranks on a one-GPU box (--dist-backend gloo), never on a full node
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":  # RCCL
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    w_all = synthetic.WORKLOADS[args.config]
    w = synthetic.shard(w_all, world)
    w_gen = w
    if args.exchange:
        # unpartitioned input: the stream spans every key; this rank's slab
        # holds the keys it owns (slot s -> rank s % world, local slot s // world)
        w_gen = synthetic.Workload(**{**w_all.__dict__, "step_swipes": w.step_swipes})
        w = synthetic.Workload(**{**w.__dict__, "n_keys": -(-w_all.n_keys // world)})
    n = args.batch or w.step_swipes
    engine = SketchEngine(local)
    stream = torch.cuda.Stream()  # a dedicated stream shared by libsketch and torch
    torch.cuda.set_stream(stream)
    engine.set_stream(stream.cuda_stream)
    for name, val in (("tile", args.tile), ("ablate", args.ablate), ("part_sub", args.part_sub)):
        if val:
            engine.set_option(name, val)
    if args.variant >= 0:
        engine.set_option("variant", args.variant)
    if args.hll_mode >= 0:
        engine.set_option("hll_mode", args.hll_mode)
    if args.pb_pairs >= 0:
        engine.set_option("pb_pairs", args.pb_pairs)
    if args.pa_tile >= 0:
        engine.set_option("pa_tile", args.pa_tile)
    if args.pa_precheck >= 0:
        engine.set_option("pa_precheck", args.pa_precheck)
    for kv in args.opt:
        name, _, val = kv.partition("=")
        engine.set_option(name, int(val))

    # Bloom preload (replicated on every rank), this rank's HLL key shard, and
    # 64 spare slots for the verification batch
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w_gen)
    t0 = time.perf_counter()
    engine.preload(0, p, w.n_members)
    preload_s = time.perf_counter() - t0
    engine.hll_reserve(w.n_keys + 64)
    variant = engine.variant(0)
    lds_k1 = variant == 1
    persistent = bool(args.persistent if args.persistent >= 0 else lds_k1) and not args.exchange
    if lds_k1:
        engine.set_option("k1_persistent", 1 if persistent else 0)
    streams_n = 1 if persistent else (args.streams or (16 if lds_k1 else 1))
    use_graph = 0 if persistent else (args.graph if args.graph >= 0 else (1 if lds_k1 else 0))
    if args.k1_grid < 0:
        cus = torch.cuda.get_device_properties(local).multi_processor_count
        args.k1_grid = cus // 2 if (lds_k1 and streams_n > 1) else 0
    if args.k1_grid:
        engine.set_option("k1_grid", args.k1_grid)

    nb = max(1, min(args.max_batches, args.steps + args.warmup))
    batches = [engine.swipe_batch(p, (rank * nb + j) * n, n) for j in range(nb)]
    out = DeviceBuffer(engine.ctx, n)  # BF.EXISTS answers (the reference stores is_valid)
    probes, nvalid = engine.swipes_stats(0, batches[0])
    width = synthetic.id_width(w)
    fixed = args.layout == "fixed"
    streams = [stream] + [torch.cuda.Stream() for _ in range(max(0, streams_n - 1))]

    ex, xviews = None, []
    if args.exchange:
        from rtsas_amd.distributed import SwipeExchange, engine_k1

        def tview(ptr, shape, typestr):  # zero-copy torch view of a library buffer
            class _V:
                __cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False),
                                            "version": 3, "strides": None}
            return torch.as_tensor(_V(), device=dev)
        ex = SwipeExchange(rank, world, engine_k1(engine), engine=engine)
        xviews = [(tview(b.bytes.ptr, (n, width), "|u1"), tview(b.slot.ptr, (n,), "<i4")) for b in batches]

    def step(j):
        if ex is not None:
            ex.swipes(*xviews[j % nb])
            return
        if len(streams) > 1:
            engine.set_stream(streams[j % len(streams)].cuda_stream)
        if fixed:
            engine.swipes_fixed_async(0, batches[j % nb], out)
        else:
            engine.swipes_async(0, batches[j % nb], out)

    if persistent:  # the same call shape as the timed region (loads the kernel)
        engine.swipes_many_async(0, [batches[j % nb] for j in range(max(1, args.warmup))],
                                 [out] * max(1, args.warmup), fixed=fixed)
    else:
        for j in range(args.warmup):
            step(j)
    engine.set_stream(stream.cuda_stream)
    torch.cuda.synchronize()
    engine.check_errors()
    graph = None
    if use_graph and len(streams) == 1:
        graph = engine.capture(lambda: [step(args.warmup + j) for j in range(args.steps)])
    elif use_graph:
        engine.swipes_many_async(0, [], branches=len(streams))  # side streams, before capture
        torch.cuda.synchronize()
        graph = engine.capture(lambda: engine.swipes_many_async(
            0, [batches[(args.warmup + j) % nb] for j in range(args.steps)],
            [out] * args.steps, branches=len(streams), fixed=fixed))
    timing = bool(args.pass_timing) and graph is None
    engine.set_option("pass_timing", 1 if timing else 0)
    engine.pass_times(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    if graph is not None:
        graph.launch()
    elif persistent:
        engine.swipes_many_async(0, [batches[(args.warmup + j) % nb] for j in range(args.steps)],
                                 [out] * args.steps, fixed=fixed)
    else:
        for s_ in streams[1:]:
            s_.wait_stream(stream)
        for j in range(args.steps):
            step(args.warmup + j)
        engine.set_stream(stream.cuda_stream)
        for s_ in streams[1:]:
            stream.wait_stream(s_)
    e1.record(stream)
    host_enqueue = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    engine.set_option("pass_timing", 0)
    engine.check_errors()  # an out-of-range slot in any timed step raises here
    step_ms = e0.elapsed_time(e1) / args.steps
    pt = engine.pass_times(reset=True)
    if world > 1:
        t = torch.tensor([elapsed, step_ms] + [ms for ms, _ in pt], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, step_ms = float(t[0]), float(t[1])
        pt = [(float(t[2 + i]), c) for i, (_, c) in enumerate(pt)]

    ms_per_step = elapsed * 1e3 / args.steps
    value = world * n * args.steps / elapsed
    cus = torch.cuda.get_device_properties(local).multi_processor_count
    alg = pass_bytes(n, nvalid, probes, width, fixed, chain_geometry(engine), lds_k1=lds_k1,
                     slab_bytes=(w.n_keys + 64) * 16384, cus=cus)
    passes = {}
    for i, (ms, cnt) in enumerate(pt):
        if cnt:
            mean = ms / cnt
            name = PASS_NAMES[i]
            # a persistent launch covers several steps and stages the filter once
            ab = (alg[name] * (args.steps / cnt if (persistent and name == "k1") else 1)
                  + (alg["k1_stage"] if name == "k1" else 0))
            passes[name] = {"ms": mean, "launches": cnt, "alg_bytes": ab,
                            "GBps": ab / (mean * 1e-3) / 1e9}
    if passes:
        dom = max(passes, key=lambda k: passes[k]["ms"])
        kern_ms, dom_bytes = passes[dom]["ms"], passes[dom]["alg_bytes"]
    else:  # graph replay: the launch time is the replay's events / steps
        dom, kern_ms, dom_bytes = "k1", step_ms, alg["k1"] + alg["k1_stage"]
    achieved = dom_bytes / (kern_ms * 1e-3) / 1e9
    # HBM-side bytes per launch of that kernel from the committed rocprofv3 PMC
    # passes of this workload (FETCH_SIZE + WRITE_SIZE, separate passes), or null
    traffic, traffic_src, pmc = None, None, None
    pmc_path = os.path.join(ROOT, "profiles", f"r02_pmc_{args.config}_{dom}.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        traffic = pmc.get("hbm_bytes_per_dispatch")
        if traffic is not None and persistent and dom == "k1":
            traffic *= args.steps / passes["k1"]["launches"] / pmc.get("steps_per_dispatch", args.steps)
        traffic_src = os.path.relpath(pmc_path, ROOT)
    roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                "kernel": dom, "kernel_ms": kern_ms, "alg_bytes_per_launch": dom_bytes,
                "device_ms_per_step": step_ms, "probes_per_swipe": probes / n,
                "valid_frac": nvalid / n, "passes": passes}
    if dom == "k_part_c":
        sectors = nvalid / (kern_ms * 1e-3) / 1e9
        roofline["random_sector_bound"] = {
            "what": "one 64-B HBM sector per valid swipe's register, against the measured random "
                    "4-B read rate over a 1.6 GB table (tools/randbench.hip)",
            "achieved_Gsectors_per_s": sectors, "peak_Gsectors_per_s": RANDOM_SECTOR_GPS,
            "frac": sectors / RANDOM_SECTOR_GPS}
        if pmc and "TCC_EA0_ATOMIC_sum" in pmc.get("mean", {}):
            # every register touch is one random 64-B request: the valid swipes'
            # pre-check loads plus the raising CASes (memory-side atomics, PMC)
            req = (nvalid + pmc["mean"]["TCC_EA0_ATOMIC_sum"]) / (kern_ms * 1e-3) / 1e9
            roofline["random_sector_bound"].update({
                "what": "random 64-B requests into the 1.6 GB register slab per second: one "
                        "pre-check load per valid swipe plus one memory-side CAS per raise "
                        "(TCC_EA0_ATOMIC_sum, PMC per dispatch), against the measured random 4-B "
                        "read rate over a 1.6 GB table (tools/randbench.hip)",
                "achieved_Gsectors_per_s": req, "frac": req / RANDOM_SECTOR_GPS,
                "loads_only_frac": sectors / RANDOM_SECTOR_GPS})
            cas = pmc["mean"]["TCC_EA0_ATOMIC_sum"] / (kern_ms * 1e-3) / 1e9
            roofline["binding"] = {
                "counter": "TCC_EA0_ATOMIC_sum",
                "what": "register CASes (memory-side device atomics, PMC per dispatch) / this run's "
                        "kernel time, against the measured rate of the same load + raising CAS "
                        "over a 1.6 GB table (tools/casbench.hip, profiles/r02_casbench.json)",
                "atomics_per_dispatch": pmc["mean"]["TCC_EA0_ATOMIC_sum"],
                "achieved_G_per_s": cas, "peak_G_per_s": RANDOM_CAS_GPS, "frac": cas / RANDOM_CAS_GPS}
    if dom == "k1" and pmc and "SQ_INSTS_VALU" in pmc.get("mean", {}):
        m = pmc["mean"]
        roofline["binding"] = {
            "counter": "SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_VALU",
            "what": "the LDS K1 is issue/latency bound, not HBM bound: per wave, the share of its "
                    "cycles waiting in s_waitcnt and issuing VALU (PMC of this workload's dispatch)",
            "wait_frac": m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"],
            "valu_frac": m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"],
            "valu_wave_insts_per_64_swipes":
                m["SQ_INSTS_VALU"] / max(1.0, pmc.get("swipes_per_dispatch", 0) / 64),
            "lds_bank_conflict_rate": pmc.get("lds_bank_conflict_rate")}
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "swipes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (device counter-based generator, seed %d)" % w.seed,
        "config": {"workload": w.name, "swipes_per_step": n, "students": w.n_members,
                   "hll_keys_total": w_all.n_keys, "hll_keys_per_gpu": w.n_keys,
                   "invalid_frac": w.invalid_frac,
                   "bloom": {"error": w.bf_error, "capacity": w.bf_capacity},
                   "id_bytes": width, "parallelism": f"dp{world} (key-sharded, Bloom replicated)",
                   "k1_variant": {0: "global-bloom", 1: "lds-bloom", 2: "xcd-regions",
                                  3: "partitioned"}[variant],
                   "layout": args.layout, "streams": len(streams),
                   "input": ("unpartitioned: alltoallv to the key owners per step"
                             if args.exchange else "routed to the key owners at ingest"),
                   "launch": ("hip-graph" if graph is not None else
                              ("persistent (one K1 launch per 48 steps)" if lds_k1 else
                               "one many-batch call (pass C of a step beside passes A/B of the next)")
                              if persistent else "host"),
                   "answers": "written (1 B per swipe)"},
        "roofline": roofline,
        "preload_s": preload_s,
        "host_enqueue_us_per_step": host_enqueue * 1e6 / args.steps,
    }
    want_cpu = rank == 0 and world == 1 and not args.no_cpu and args.cpu_seconds > 0
    if not args.no_check or want_cpu:
        orc = ge.load_oracle()
        chain = oracle_chain(engine, orc, w, p)
        if not args.no_check:
            line["check"] = verify(engine, orc, chain, w, rank, world, dist, dev)
        if want_cpu:
            line["cpu_baseline"] = cpu_baseline(orc, chain, w, batches[0], args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if graph is not None:
        graph.free()
    for b in batches:
        b.free()
    out.free()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
