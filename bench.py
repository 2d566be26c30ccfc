"""Benchmark of the fused validate-and-count hot path (K1: BF.EXISTS +
valid-gated PFADD) -- BASELINE.json's metric on its north-star configuration.

Default workload: C3 (configs[2], the configuration BASELINE.md quotes the
1/2/4/8-GPU curve on), this rank's shard of it: the replicated 10M-student
Bloom filter (RESERVE 0.001 / 1e7: 19.8 MB, k = 11) preloaded by BF.MADD, a
Zipf(1.1)-over-lectures x uniform-over-days stream of 8-digit ids with 10 %
invalid swipes, and the HLL keys this rank owns (distributed.KeyMap:
MurmurHash64A(key name) mod world over the 100k README-form key names; all
of them at N = 1, ~12.5k per rank at N = 8).  One step = one K1 call over
one resident batch of 2^28 swipes per GPU (C3's 1B-swipe stream in 4 steps;
answers written, PFADD of the valid ones): the partitioned K1 in even
sub-batches of 2^25 swipes (sketch_part.hip: hash + probe records,
LDS-slice probes, answers + the segmented PFADD's records and level-2 sort),
then one window pass of the segmented PFADD over the slab (each key window
staged in LDS, raised, its risen lines flushed).  `--config c2` runs C2 (1M
swipes, the LDS K1).

Inputs are generated on the GPU and resident in HBM before timing; every
step consumes a distinct batch of the stream.  Timing: W untimed warm-up
steps, then K steps bracketed by barrier + synchronize; value = swipes of all
ranks / the slowest rank's wall time.  The timed region carries no
instrumentation.  Per-kernel times for the roofline come from a separate
REPLAY of the same steps: the register slab is zeroed, the W warm-up steps
are re-run, and the K steps are replayed with a HIP event pair around every
K1 kernel on the stream it runs on (ske_pass_times) -- the same batches from
the same register state, so the same work.

`secondary` (N = 1, default workload): C2 (configs[1], the configuration
sized for one MI355X) measured in the same process on its own context.

N>1: one process per GPU (torch.distributed.run), RCCL ("nccl") process
group; every rank runs its own stream over its own key shard with the Bloom
replicated (no data-path collective; weak scaling).  After timing, every rank
checks a verification stream through the SHIPPED classes: the stream names
64 keys of a second universe (distributed.KeyMap), each rank runs K1 on the
swipes of the keys it owns (or, with --exchange 1, routes its slice through
distributed.SwipeExchange), and distributed.ShardedSketch answers union
PFCOUNT, PFCOUNT of every key and a rollup by key name over RCCL; answers,
registers and every query are compared with the CPU oracle over the whole
stream ("check").

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
HBM_MEASURED_GBS = 6290.0  # MI355X_MICROARCH.md: measured streaming read rate
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
PASS_NAMES = ["k1", "k_part_a", "k_part_b", "k_part_c", "k_seg_d", "k_seg_e", "feed_h2d", "feed_d2h", "feed_call"]
K1_PASSES = 6  # PASS_NAMES[:6] are K1 kernels; the rest the stages of a host-fed call
PMC_ROUNDS = ["r06", "r05", "r04", "r03", "r02"]  # newest committed PMC summaries first
VERIFY_KEYS = 64
# swipes per GPU and step where it differs from the workload's own
# step_swipes: C3 takes 2^28 since round 6 (its 1B-swipe stream in 4 steps;
# 2^27 in round 5, 16 M before).  The segmented PFADD streams each key window
# of the slab once per step, ~0.64 ms whatever the step, so the step is sized
# to many register updates per slab line: per 2^27 swipes the window pass
# costs 0.85 ms at a 2^27 step and 0.53 ms at 2^28
BENCH_STEP = {"c3": 1 << 28}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment and N > 1, "
                         "bench.py launches the N ranks itself (torch.distributed.run)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--secondary", default="auto",
                    help="config measured after the headline in the same process (N = 1 only); "
                         "auto = c2 when the headline is c3, none = skip")
    ap.add_argument("--batch", type=int, default=0, help="swipes per step (default: config)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--tile", type=int, default=0, help="K1 swipes per thread in flight (1,2,4,8)")
    ap.add_argument("--variant", type=int, default=-1,
                    help="-1 auto, 0 global Bloom, 1 LDS Bloom, 2 XCD-partitioned, 3 partitioned")
    ap.add_argument("--max-batches", type=int, default=64)
    ap.add_argument("--part-sub", type=int, default=0,
                    help="partitioned K1: swipes per sub-batch of its three passes (0 = default)")
    ap.add_argument("--exchange", type=int, default=0,
                    help="1 = unpartitioned input: every rank's batches span ALL keys and a step "
                         "routes them to the key owners with all_to_all_single "
                         "(distributed.SwipeExchange), runs K1 there and returns the answers; "
                         "step j+1's routing and forward exchange overlap step j's K1 (2 = the "
                         "one-stream form, for A/B)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="library option (ske_set_option), e.g. k1_grid=128; repeatable")
    ap.add_argument("--persistent", type=int, default=-1,
                    help="1 = the K timed steps as ONE ske_swipes_many_async call (for the LDS "
                         "K1 one persistent launch over the K batches; the default for the LDS K1); "
                         "0 = a K1 launch per step")
    ap.add_argument("--streams", type=int, default=0,
                    help="HIP streams / graph branches the steps alternate over (0: 16 for the "
                         "LDS K1, 1 otherwise)")
    ap.add_argument("--k1-grid", type=int, default=-1, help="blocks of the short-id LDS K1")
    ap.add_argument("--graph", type=int, default=-1,
                    help="1 = record the K timed steps into a HIP graph and replay it (default for "
                         "the LDS K1); 0 = launch them from the host (default otherwise)")
    ap.add_argument("--pass-replay", type=int, default=1,
                    help="1 = per-kernel times from an instrumented replay of the same steps "
                         "after the timed region (the timed region itself is never instrumented)")
    ap.add_argument("--sync-spin", type=int, default=1,
                    help="1: the HIP runtime spins instead of yielding while the host waits for the "
                         "device (hipDeviceScheduleSpin, set before the device is initialised)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N>1 (nccl = RCCL over xGMI; gloo only to rehearse "
                         "several ranks on a one-GPU box)")
    ap.add_argument("--layout", default="offsets", choices=["offsets", "fixed"],
                    help="id batch layout: bytes + u32 offsets, or fixed-width ids")
    ap.add_argument("--shares", default="mass", choices=["mass", "equal"],
                    help="N > 1, input routed at ingest: mass = one global stream of N x the "
                         "config's step swipes, each rank's batch the probability mass of the keys "
                         "it owns (the fixed 1B-event stream of north_star, cut per step); "
                         "equal = every rank the config's step swipes over its own keys")
    ap.add_argument("--ownership", default="hash", choices=["hash", "mass"],
                    help="N > 1: key owners by MurmurHash64A(key) mod N (north_star's rule, the default) or "
                         "mass-balanced (distributed.balanced_owners: the key hash's 256 x N virtual buckets "
                         "assigned to ranks by greedy key mass)")
    ap.add_argument("--rollup", type=int, default=-1,
                    help="1: after the K1 steps, time the rankings / campus PFMERGE over the registers "
                         "(ShardedSketch; default on for --config c5)")
    ap.add_argument("--stream-1b", type=int, default=1,
                    help="1: after timing, north_star's 1B-event stream from a zeroed slab: ceil(2^30 / "
                         "swipes per step of all ranks) steps (8 at N = 1), timed, then replayed with "
                         "per-pass events (stream_1b; host-launched partitioned K1 only)")
    ap.add_argument("--host-fed", type=int, default=1,
                    help="N = 1: also time one 16M-swipe sample handed over in host memory (PCIe-inclusive, "
                         "pageable / pinned / fixed-width 1-bit answers), reported as host_fed, never value")
    ap.add_argument("--shard", type=int, default=0,
                    help="N > 0: run ONE rank's share of an N-rank job on this GPU (its owned keys and, "
                         "with --shares mass, its batch), to measure the per-GPU work of the N-GPU "
                         "configuration on one GPU; no collective (the line keeps n_gpus 1)")
    ap.add_argument("--shard-rank", type=int, default=-1,
                    help="with --shard: the rank simulated (-1 = the one owning the most key mass)")
    a = ap.parse_args(argv)
    if a.shard and a.exchange:
        ap.error("--shard simulates owner-routed input only")
    return a


def free_port():
    """A TCP port on 127.0.0.1 nothing listens on (the rendezvous port of a
    self-launched multi-rank run)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(args, argv, env):
    """How this invocation runs (the driver's contract: `bench.py --gpus N` is
    N ranks, one per GPU).

    - WORLD_SIZE set (an external torch.distributed.run): this process is one
      rank; --gpus, when given, must equal WORLD_SIZE.  Returns None.
    - WORLD_SIZE unset and --gpus N > 1: returns the command that launches the
      N ranks (torch.distributed.run on 127.0.0.1, the same bench arguments);
      the caller runs it as a child process BEFORE anything touches the GPU
      and exits with its status.  Rank 0 prints the JSON line.
    - otherwise one rank in this process (None)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if args.gpus is not None and int(ws) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
        return None
    n = args.gpus or 1
    if n <= 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={free_port()}",
            os.path.abspath(__file__), *argv]


def rank_swipes(step_swipes, mass, world, mode):
    """Swipes this rank processes per step.  `mass`: the probability mass of
    the keys it owns in the global stream.  mass mode: this rank's share of a
    global step of world x step_swipes swipes; equal mode: step_swipes."""
    if world <= 1 or mode == "equal":
        return step_swipes
    return max(1, int(round(world * step_swipes * mass)))


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


def part_sub_default(geom):
    """The partitioned K1's default sub-batch (sketch_part.hip part_sub): 2^25
    swipes, or less where the probe records of one of the 8 XCD tile groups
    (tiles of 1024 swipes, k-sum * 1024 4-B records per tile rounded to 32)
    would pass a 2^31-byte range."""
    ksum = sum(k for _, k in geom)
    stride = ((ksum << 10) + 31) & ~31
    tiles = ((1 << 31) - 1) // (stride * 4)
    return min(1 << 25, (tiles - 8) * 8 * 1024)


def oracle_chain(engine, orc, w, p):
    """The Bloom chain as the oracle builds it from the same preload (RedisBloom
    SBChain_Add restated, oracle/sketch_oracle.c) -- test infrastructure."""
    mb = engine.members_batch(p, 0, w.n_members)
    buf, offs, _ = mb.to_host()
    mb.free()
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    chain.madd_packed(buf, offs)
    return chain


def cpu_baseline(orc, chain, w, b0, seconds, key_name):
    """The processor loop attendance_processor.py:100-137 (BF.EXISTS, then
    PFADD when valid) on the host, over a bounded sample of the first batch:
      - the C oracle on all host threads (orc_process_swipes_mt; the value),
        and on one thread;
      - the reference's per-event Python loop (json.loads, fromisoformat,
        BF.EXISTS, PFADD per message) over the oracle, one core (§8d item 1)."""
    import numpy as np
    from datetime import datetime
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
        _, _, lecture, day = key_name(int(slot[i])).split(":")
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


def host_fed(engine, batch, reps=5, cap=1 << 24):
    """SURVEY §7 item 8 / DESIGN §4: the PCIe-inclusive rate -- the same
    swipes handed over in HOST memory (the reference's loop is fed from the
    host, attendance_processor.py:101-113): ske_swipes(..., SKE_MEM_HOST)
    stages ids, offsets and slots host -> device, runs K1 and copies the
    answers back; ske_swipes_fixed_bits the fixed-width form with 1-bit
    answers.  Pageable numpy and pinned torch buffers; median of `reps`
    synchronous calls over the first min(n, cap) swipes of the batch.  Never
    `value` (that one starts with the batch resident in HBM).  Answers are
    compared with the device-resident call's."""
    import numpy as np
    import torch
    from rtsas_amd._lib import SKE_MEM_HOST
    from rtsas_amd.engine import DeviceBuffer
    buf, offs, slot = batch.to_host()
    n = min(len(offs) - 1, cap)
    width = int(offs[1] - offs[0])
    fixed = bool(np.all(np.diff(offs[:n + 1]) == width))
    buf = np.ascontiguousarray(buf[:int(offs[n]) + 16])
    offs = np.ascontiguousarray(offs[:n + 1])
    slot = np.ascontiguousarray(slot[:n].astype(np.uint32))
    ref = DeviceBuffer(engine.ctx, n)
    ptr = lambda a: C.c_void_p(a.ctypes.data if isinstance(a, np.ndarray) else a.data_ptr())
    engine.ctx.call("ske_swipes", 0, C.c_void_p(batch.slot.ptr), C.c_void_p(batch.bytes.ptr),
                    C.c_void_p(batch.offs.ptr), n, C.c_void_p(ref.ptr), 1)  # SKE_MEM_DEVICE
    want = ref.to_host(np.uint8, n)
    ref.free()

    stages = {}

    def timed(call):
        """median wall time of `reps` calls after one untimed call, and per
        call its stages: the HIP events the library records on the streams
        each stage runs on (H2D copies, the K1 kernels, D2H copies, the whole
        call), so that a slow call shows which stage was slow; `stages`
        holds the median call's and the slowest call's"""
        # the untimed call runs with the events on too, so the library's event
        # pool is filled before timing (creating ~60 events inside the first
        # timed call had made it look 2.4x slower in its H2D stage)
        engine.set_option("pass_timing", 1)
        call()
        engine.pass_times(reset=True)
        ts, per = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
            pt = engine.pass_times(reset=True)
            per.append({"wall_ms": ts[-1] * 1e3, "h2d_ms": pt[6][0], "k1_ms": sum(ms for ms, _ in pt[:6]),
                        "d2h_ms": pt[7][0], "call_ms": pt[8][0], "chunks": pt[6][1]})
        engine.set_option("pass_timing", 0)
        order = np.argsort(ts)
        stages.clear()
        stages.update({"median_call": per[int(order[len(ts) // 2])], "slowest_call": per[int(order[-1])],
                       "wall_ms_all": [round(t * 1e3, 3) for t in ts]})
        return float(np.median(ts))

    out = {"swipes": n, "what": "ske_swipes(..., SKE_MEM_HOST): H2D of ids + offsets + slots, K1, D2H of the "
                                "answers, synchronous; median of %d calls; stages: device-side HIP events per "
                                "stage (h2d: the copies' span on the stream they run on, summed over chunks; "
                                "k1: the kernels; d2h; call: first enqueued operation to the last) of the "
                                "median and the slowest call" % reps}

    def offsets_form(b, o, sl, ans, label):
        t = timed(lambda: engine.ctx.call("ske_swipes", 0, ptr(sl), ptr(b), ptr(o), n, ptr(ans), SKE_MEM_HOST))
        got = ans if isinstance(ans, np.ndarray) else ans.numpy()
        out[label] = {"swipes_per_s": n / t, "ms": t * 1e3,
                      "host_GBps": (b.nbytes + o.nbytes + sl.nbytes + n) / t / 1e9,
                      "answers_equal": bool(np.array_equal(got, want)), "stages": dict(stages)}

    offsets_form(buf, offs, slot, np.zeros(n, np.uint8), "pageable")
    pb, po, ps = (torch.from_numpy(x).pin_memory() for x in (buf, offs, slot))
    pans = torch.zeros(n, dtype=torch.uint8).pin_memory()
    offsets_form(pb, po, ps, pans, "pinned")
    if fixed:
        ids = np.ascontiguousarray(buf[:n * width])
        bits = np.zeros((n + 7) // 8, np.uint8)
        pid = torch.from_numpy(ids).pin_memory()
        pbits = torch.zeros((n + 7) // 8, dtype=torch.uint8).pin_memory()
        for label, i_, s_, b_ in (("fixed_bits_pageable", ids, slot, bits), ("fixed_bits_pinned", pid, ps, pbits)):
            t = timed(lambda: engine.ctx.call("ske_swipes_fixed_bits", 0, ptr(s_), ptr(i_), width, n, ptr(b_),
                                              SKE_MEM_HOST))
            got = b_ if isinstance(b_, np.ndarray) else b_.numpy()
            out[label] = {"swipes_per_s": n / t, "ms": t * 1e3,
                          "host_GBps": (n * width + 4 * n + (n + 7) // 8) / t / 1e9,
                          "answers_equal": bool(np.array_equal(np.unpackbits(got, count=n, bitorder="little"),
                                                               want)), "stages": dict(stages)}
    return out


def rollup_bench(run, dist, reps=3):
    """C5's query side after the K1 steps (attendance_analysis.py:87-97 in
    PFCOUNT form, README.md:179): through distributed.ShardedSketch
    planned queries -- PFCOUNT of every lecture-day key, the per-lecture
    union of its day keys (K2 per group at N = 1; K3 + reduce_scatter MAX +
    K2 at N > 1), the campus-wide PFMERGE of every key, and the top / bottom-3
    lectures.  Best of `reps` after one untimed call; wall time around each
    query (host staging included).  Checked against the oracle's estimator
    (oracle hll_count_regs) over the device registers of sampled lectures and
    keys, and of the campus union recomputed with torch amax."""
    import numpy as np
    import torch
    import rtsas_amd
    from rtsas_amd.distributed import ShardedSketch
    from rtsas_amd.processor import rank_top_bottom_dev
    w = run.w_all
    L, D = w.zipf_lectures, w.zipf_days
    world, rank, dev = run.world, run.rank, run.dev
    client = rtsas_amd.SketchClient(context=run.engine.ctx)
    sk = ShardedSketch(client, rank, world)
    km = run.km
    groups = [np.arange(l * D, (l + 1) * D) for l in range(L)]
    plan = sk.plan(km, groups)
    allk = np.arange(len(km))
    kplan = sk.plan_keys(km, allk)
    scratch = run.sinks[0 if run.args.shard else run.kr] + 1

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def timed(fn):
        out = fn()
        best = 1e30
        for _ in range(reps):
            barrier()
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        t = torch.tensor([best], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0]), out

    # every query device-resident: the plans' slot lists live on the device,
    # counts stay there, and only the top / bottom-3 (6 keys) reach the host
    t_each, each_dev = timed(lambda: sk.pfcount_each_planned(kplan))
    t_rank_each, (ehead, etail) = timed(lambda: rank_top_bottom_dev(each_dev, 3))
    t_groups, lect_dev = timed(lambda: sk.rollup_planned(plan, device=True))
    t_merge, (campus, row) = timed(lambda: sk.pfmerge_planned(kplan, scratch))
    t_rank, (head, tail) = timed(lambda: rank_top_bottom_dev(lect_dev, 3))
    names = [f"LECT{l:05d}" for l in range(L)]
    each = each_dev.cpu().numpy().astype(np.uint64)  # (the checks' copies, after timing)
    lect = lect_dev.cpu().numpy().astype(np.uint64)
    # ---- checks: the oracle's estimator over the device registers
    orc = __import__("__graft_entry__").load_oracle()
    p_, nb = C.c_void_p(), C.c_uint64()
    run.engine.ctx.call("ske_hll_slab", C.byref(p_), C.byref(nb))
    nmine = km.count(run.kr)

    class _V:
        __cuda_array_interface__ = {"shape": (max(1, nmine), 16384), "typestr": "|u1", "data": (p_.value, False),
                                    "version": 3, "strides": None}
    slab = torch.as_tensor(_V(), device=dev)
    cdev = dev if dist.is_initialized() and dist.get_backend() == "nccl" else "cpu"

    def global_max(rows):
        t = rows.to(cdev) if cdev == "cpu" else rows
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.cpu().numpy()

    ok_l = True
    for l in sorted({0, 1, L // 2, L - 1}):
        g = groups[l]
        mine = g[km.owner[g] == rank]
        r = slab[torch.from_numpy(km.local[mine].astype(np.int64)).to(dev)].amax(0) if mine.size else \
            torch.zeros(16384, dtype=torch.uint8, device=dev)
        ok_l &= orc.hll_count_regs(global_max(r.reshape(1, -1))[0]) == int(lect[l])
    rng = np.random.default_rng(11)
    sample = rng.choice(len(km), size=64, replace=False)
    want = np.zeros(64, np.int64)
    for i, g in enumerate(sample):
        if km.owner[g] == rank:
            want[i] = orc.hll_count_regs(slab[int(km.local[g])].cpu().numpy())
    wt = torch.from_numpy(want)
    if world > 1:
        wt = wt.to(cdev)
        dist.all_reduce(wt, op=dist.ReduceOp.SUM)
    ok_e = bool(np.array_equal(wt.cpu().numpy().astype(np.uint64), each[sample]))
    u = torch.zeros(16384, dtype=torch.uint8, device=dev)
    for a in range(0, nmine, 1 << 16):
        u = torch.maximum(u, slab[a:min(nmine, a + (1 << 16))].amax(0))
    ug = global_max(u.reshape(1, -1))[0]
    ok_m = bool(np.array_equal(ug, row.cpu().numpy()[0])) and orc.hll_count_regs(ug) == campus
    order = np.lexsort((np.arange(L), ~lect))
    ok_r = list(head) == [int(i) for i in order[:3]] and list(tail) == [int(i) for i in order[-3:]]
    # the lecture-day ranking: key index order is the key names' order (LECT%05d:YYYY-MM-DD)
    knames = np.asarray(run.names)
    eorder = np.lexsort((np.arange(len(km)), ~each))
    ok_re = bool(np.all(knames[:-1] < knames[1:])) and list(ehead) == [int(i) for i in eorder[:3]] and \
        list(etail) == [int(i) for i in eorder[-3:]]
    ok = torch.tensor([int(ok_l and ok_e and ok_m and ok_r and ok_re)], device=cdev)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    slab_rank = nmine * 16384
    return {"each_ms": t_each * 1e3, "groups_ms": t_groups * 1e3, "merge_ms": t_merge * 1e3,
            "rank_ms": t_rank * 1e3, "rank_each_ms": t_rank_each * 1e3, "ok": bool(ok.item()),
            "checks": {"sampled_lecture_unions": bool(ok_l), "sampled_key_counts": ok_e,
                       "campus_pfmerge": ok_m, "top_bottom_3": ok_r, "top_bottom_3_day_keys": ok_re},
            "keys": len(km), "lectures": L, "days": D, "slab_GB_this_gpu": slab_rank / 1e9,
            "GBps_this_gpu": {"each": slab_rank / t_each / 1e9, "groups": slab_rank / t_groups / 1e9,
                              "merge": slab_rank / t_merge / 1e9},
            "campus_pfcount": campus, "top3": {names[i]: int(lect[i]) for i in head},
            "bottom3": {names[i]: int(lect[i]) for i in tail},
            "top3_day_keys": {run.names[i]: int(each[i]) for i in ehead},
            "bottom3_day_keys": {run.names[i]: int(each[i]) for i in etail},
            "what": "ShardedSketch planned queries over this run's registers, device-resident (plans built "
                    "once on the device, counts kept there, top / bottom-3 by rank_top_bottom_dev: 6 keys "
                    "reach the host); wall time per query, best of %d; checked with the oracle's estimator "
                    "over device registers and a full host sort" % reps}


def stream_1b(run, n_all, warm_pt, total=1 << 30):
    """north_star's workload as a whole: the 1B-event stream
    from a zeroed slab -- ceil(2^30 / n_all) steps of this run's batches
    (0, 1, ...; 4 steps of 2^28 at N = 1, the whole stream on every rank's
    share at N > 1), timed like the headline (barrier + synchronize on both
    sides, max over ranks), then the same cold stream replayed with a HIP
    event pair around every kernel for the per-pass split.  `warm_pt`: the
    headline's instrumented replay (steps W..W+K-1 of the stream on a slab
    warmed by W steps), for the cold-versus-warm comparison per pass."""
    import torch
    a, e, dist, world = run.args, run.engine, run.dist, run.world
    steps = -(-total // n_all)

    def go(instrument):
        run.zero_slab()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        if instrument:
            e.set_option("pass_timing", 1)
            e.pass_times(reset=True)
        t0 = time.perf_counter()
        for j in range(steps):
            run.step(j)
        if run.ex is not None:
            run.ex.flush()
        e.set_stream(run.stream.cuda_stream)
        torch.cuda.synchronize()
        run.finish()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        pt = None
        if instrument:
            pt = e.pass_times(reset=True)
            e.set_option("pass_timing", 0)
        e.check_errors()
        return el, pt

    el, _ = go(False)
    if world > 1:
        cdev = run.dev if a.dist_backend == "nccl" else "cpu"
        t = torch.tensor([el], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
    _, pt = go(True)

    def per_pass(p, nsteps):
        return {PASS_NAMES[i]: {"ms": ms / c, "launches": c, "ms_per_step": ms / nsteps}
                for i, (ms, c) in enumerate((p or [])[:K1_PASSES]) if c}
    cold, warm = per_pass(pt, steps), per_pass(warm_pt, a.steps)
    return {"swipes": steps * n_all, "steps": steps, "swipes_per_s": steps * n_all / el,
            "ms_per_step": el * 1e3 / steps, "wall_s": el,
            "passes": cold, "passes_warm": warm,
            "cold_minus_warm_ms_per_step": {k: cold[k]["ms_per_step"] - warm[k]["ms_per_step"]
                                            for k in cold if k in warm},
            "what": "the first %d swipes of the stream (batches 0..%d) from a zeroed slab, every step's "
                    "registers raised from cold; passes: per-kernel HIP events of a replay of the same "
                    "cold stream; passes_warm: the headline's replay (steps %d..%d after %d warm-up "
                    "steps)" % (steps * n_all, steps - 1, a.warmup, a.warmup + a.steps - 1, a.warmup)}


def checked(fn, *a, **k):
    """A check that raises is reported in the line (ok false, the error), not
    by losing the measured line: every rank runs the same checks on the same
    shapes, so an error (an unsupported collective, a shape mismatch) is raised
    on every rank alike before the next collective."""
    try:
        return fn(*a, **k)
    except Exception as e:  # noqa: BLE001 - reported, not swallowed
        print(f"CHECK ERROR {fn.__name__}: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        return {"ok": False, "error": f"{type(e).__name__}: {e}"[:400]}


def verify(engine, orc, chain, w, km, rank, world, dist, dev, exchange, sinks, prefix="VERIFY", under=None):
    """The shipped multi-GPU classes on a verification stream, against the
    CPU oracle over the WHOLE stream (no collective on the expected side).

    The stream (identical on every rank: same seed, generated on the device)
    names VERIFY_KEYS keys of a second universe, `vk`, bound above this rank's
    workload keys (KeyMap base = the workload map's slots_end).  Pre-routed
    input: each rank runs K1 on the swipes of the keys it owns (ingest
    routing by owner()); --exchange: each rank hands its slice of the stream
    to distributed.SwipeExchange.  Then distributed.ShardedSketch, over a
    client that KeyMap.bind named, answers union PFCOUNT, PFCOUNT of every key
    and a rollup (RCCL at N > 1).  `under`: a KeyMap whose slots the
    verification keys go above (default: the workload's).  `sinks`: every
    rank's spare slot for SwipeExchange.swipes_async's padding."""
    import numpy as np
    import torch
    import rtsas_amd
    from rtsas_amd import synthetic
    from rtsas_amd.distributed import KeyMap, ShardedSketch, SwipeExchange, engine_k1
    from rtsas_amd.engine import DeviceBatch, DeviceBuffer
    names = [f"hll:unique:{prefix}{j:03d}:2025-10-03" for j in range(VERIFY_KEYS)]
    under = km if under is None else under
    vk = KeyMap(names, world, base=[under.slots_end(r) for r in range(world)])
    engine.hll_reserve(vk.slots_end(rank))
    client = rtsas_amd.SketchClient(context=engine.ctx)
    vk.bind(client, rank)
    wv = synthetic.Workload(**{**w.__dict__, "n_keys": VERIFY_KEYS, "zipf_lectures": 0, "zipf_days": 0})
    pv = engine.gen_params(wv, seed=w.seed + 7919, slot_base=0)
    n = 1 << 19
    b = engine.swipe_batch(pv, 0, n)
    buf, offs, gkey = b.to_host()
    width = int(offs[1] - offs[0])
    regs_o = np.zeros((VERIFY_KEYS, 16384), np.uint8)
    want, _, _ = orc.process_swipes(chain, regs_o, gkey.astype(np.uint32), buf, offs)
    want = want.astype(np.uint8)
    if exchange:
        lo, hi = rank * n // world, (rank + 1) * n // world
        ids = torch.as_tensor(buf[:n * width].reshape(n, width)[lo:hi].copy(), device=dev)
        ex = SwipeExchange(rank, world, engine_k1(engine), vk, engine=engine, sink_slots=sinks)
        # the host-free form (as the timed steps), every rank's slice <= n_max
        got = ex.swipes_async(ids, torch.as_tensor(gkey[lo:hi].astype(np.int64), device=dev),
                              n_max=-(-n // world))
        ex.settle()
        torch.cuda.synchronize()
        ok_answers = bool(np.array_equal(got.cpu().numpy(), want[lo:hi]))
    else:
        sel = np.nonzero(vk.owner[gkey] == rank)[0]
        sb = np.ascontiguousarray(buf[:n * width].reshape(n, width)[sel]).reshape(-1)
        so = np.arange(0, width * sel.size + 1, width, dtype=np.uint32)
        mb = DeviceBatch.from_host(engine.ctx, sb, so, vk.local[gkey[sel]])
        out = DeviceBuffer(engine.ctx, max(1, sel.size))
        if sel.size:
            engine.swipes(0, mb, out)
        ok_answers = bool(np.array_equal(out.to_host(np.uint8, sel.size), want[sel]))
        mb.free()
        out.free()
    b.free()
    engine.sync()
    mine = vk.keys_of(rank)
    have = engine.registers_all(vk.slots_end(rank))
    ok_regs = bool(np.array_equal(have[vk.local[mine]], regs_o[mine]))
    sk = ShardedSketch(client, rank, world)
    groups = [names[i::8] for i in range(8)] + [names, []]
    union = sk.pfcount_union(names)
    each = sk.pfcount_each(names)
    roll = sk.rollup(groups)
    ok_union = union == orc.hll_count_regs(regs_o.max(axis=0))
    ok_each = each.tolist() == [orc.hll_count_regs(r) for r in regs_o]
    ok_roll = roll.tolist() == [orc.hll_count_regs(regs_o[[names.index(k) for k in g]].max(axis=0))
                                if g else 0 for g in groups]
    ok = torch.tensor([int(ok_answers and ok_regs and ok_union and ok_each and ok_roll)],
                      device=dev if dist.is_initialized() and dist.get_backend() == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    verify.last_map = vk
    return {"ok": bool(ok.item()), "stream_swipes": n, "keys": VERIFY_KEYS, "keys_owned": int(mine.size),
            "input": "SwipeExchange.swipes_async slice" if exchange else "owner-routed",
            "answers": ok_answers, "owned_registers": ok_regs,
            "sharded_pfcount_union": bool(ok_union), "sharded_pfcount_each": bool(ok_each),
            "sharded_rollup": bool(ok_roll), "union_pfcount": int(union),
            "backend": dist.get_backend() if world > 1 else "none"}


def pass_bytes(n, nvalid, probes, width, fixed, geometry, lds_k1=False, slab_bytes=0, cus=256, seg=False,
               nsub=1):
    """Algorithmic bytes per launch of each K1 kernel: streams
    at their size, every random access at one 64-B HBM sector.  The LDS K1
    (lds_k1) reads the filter once per block (staged into LDS, probes cost no
    HBM) and its register words only when the slab does not fit on chip.
    seg: the segmented PFADD -- pass C writes a 4-B record per valid swipe
    instead of touching registers; the level-2 sort reads and writes every
    record once; the window pass reads every record and the slab once and
    writes the slab back once (its lines that rose, at most the whole slab).
    Per-launch figures of the per-sub-batch kernels are per sub-batch
    (nsub sub-batches of n / nsub swipes)."""
    s_off = 0 if fixed else 4
    ksum = sum(k for _, k in geometry)
    nslices = sum(-(-bits // (1 << 19)) for bits, _ in geometry)
    filter_bytes = sum(bits // 8 for bits, _ in geometry)
    rec = 4 * ksum * n
    ntiles = -(-n // 1024)
    # fail bytes per swipe: one per link; none for the fail-list chains (one
    # link, k = 11), whose overflow flags live in the HLL word's top byte
    nfail = 0 if (len(geometry) == 1 and ksum == 11) else len(geometry)
    return {
        # one kernel: ids + offsets + slot + answer streamed, one sector per
        # RedisBloom probe, one sector read + one written per valid swipe
        "k1": (n * (width + s_off + 4 + 1)
               + (128 * nvalid if slab_bytes > MALL_BYTES else 0)) if lds_k1 else
              n * (width + s_off + 4 + 1) + 64 * probes + 128 * nvalid,
        # the LDS K1 stages the filter into every block's LDS once per launch
        "k1_stage": filter_bytes * cus if lds_k1 else 0,
        # ids + offsets in; probe records, run table, HLL word, fail bytes out
        "k_part_a": n * (width + s_off) + rec + 4 * (nslices + 1) * ntiles + 4 * n + n * nfail,
        # probe records + their run boundaries in, the filter staged once
        "k_part_b": rec + 8 * nslices * ntiles + filter_bytes,
        # fail byte, HLL word, slot in, answer out; per valid swipe its register's
        # sector read + written (SURVEY §8d's 128·v, as the one-kernel K1 above),
        # or (seg) its 4-B record written
        "k_part_c": n * (nfail + 4 + 4 + 1) + (4 if seg else 128) * nvalid,
        "k_seg_d": 8 * nvalid,
        "k_seg_e": 4 * nvalid * nsub + 2 * slab_bytes,
    }


def load_pmc(config, kernel):
    """The newest committed rocprofv3 PMC summary of this workload's kernel."""
    for r in PMC_ROUNDS:
        path = os.path.join(ROOT, "profiles", f"{r}_pmc_{config}_{kernel}.json")
        if os.path.exists(path):
            with open(path) as f:
                return json.load(f), os.path.relpath(path, ROOT)
    return None, None


class _ShardView:
    """The slot layout of one simulated rank (--shard) as verify() sees it:
    a one-rank map whose workload slots end where the shard's do."""

    def __init__(self, end):
        self.end = end

    def slots_end(self, r):
        return self.end


class Run:
    """One workload on one context: setup, timed steps, instrumented replay."""

    def __init__(self, args, cfg, world, rank, local, dev, dist):
        import torch
        from rtsas_amd import synthetic
        from rtsas_amd.distributed import KeyMap
        from rtsas_amd.engine import DeviceBuffer, SketchEngine
        self.args, self.cfg, self.world, self.rank, self.dist, self.dev = args, cfg, world, rank, dist, dev
        self.torch = torch
        w_all = synthetic.WORKLOADS[cfg]
        self.w_all = w_all
        # the job's key universe and its one ownership rule (distributed.KeyMap)
        self.names = synthetic.key_names(w_all)
        probs = synthetic.key_probs(w_all)
        # --shard N: this process plays one rank (kr) of an N-rank job (kw)
        kw = args.shard if args.shard else world
        self.km = KeyMap(self.names, kw, balance=args.ownership, weights=probs)
        if args.shard:
            masses = [float(probs[self.km.keys_of(r)].sum()) if probs is not None
                      else self.km.keys_of(r).size / len(self.names) for r in range(kw)]
            kr = args.shard_rank if args.shard_rank >= 0 else int(max(range(kw), key=lambda r: masses[r]))
        else:
            kr = rank
        self.kw, self.kr = kw, kr
        mine = self.km.keys_of(kr)
        if args.exchange:
            # unpartitioned input: the stream spans every key (global indices);
            # this rank's slab holds the keys it owns
            w_gen = synthetic.Workload(**{**w_all.__dict__})
            cdf = None
        else:
            # routed at ingest: this rank's stream is the global stream's
            # share of the keys it owns, over their local slots
            # (a uniform workload stays uniform over the owned keys: no table)
            w_gen = synthetic.Workload(**{**w_all.__dict__, "n_keys": int(mine.size),
                                          "zipf_lectures": 0, "zipf_days": 0})
            cdf = synthetic.cdf_from_probs(probs[mine]) if probs is not None else None
        self.w = w = synthetic.Workload(**{**w_all.__dict__, "n_keys": int(mine.size)})
        # the probability mass of this rank's keys in the global stream
        self.mass = float(probs[mine].sum()) if probs is not None else mine.size / len(self.names)
        self.shares = "equal" if args.exchange else args.shares
        self.n = n = rank_swipes(args.batch or BENCH_STEP.get(cfg, w.step_swipes), self.mass, kw, self.shares)
        self.engine = engine = SketchEngine(local)
        self.stream = stream = torch.cuda.Stream()  # shared by libsketch and torch
        torch.cuda.set_stream(stream)
        engine.set_stream(stream.cuda_stream)
        for name, val in (("tile", args.tile), ("part_sub", args.part_sub)):
            if val:
                engine.set_option(name, val)
        if args.variant >= 0:
            engine.set_option("variant", args.variant)
        for kv in args.opt:
            name, _, val = kv.partition("=")
            engine.set_option(name, int(val))
        # Bloom preload (replicated on every rank) and this rank's HLL keys
        engine.reserve(0, w.bf_error, w.bf_capacity)
        self.p = p = engine.gen_params(w_gen, cdf=cdf)
        t0 = time.perf_counter()
        engine.preload(0, p, w.n_members)
        self.preload_s = time.perf_counter() - t0
        self.nslots = self.km.slots_end(kr)
        # past the workload's keys: the verification universes (verify(), up
        # to 2 x VERIFY_KEYS slots), then the exchange's sink slot (padding
        # rows of SwipeExchange.swipes_async; no key lives there)
        self.sinks = [self.km.slots_end(r) + 2 * VERIFY_KEYS for r in range(kw)]
        engine.hll_reserve(self.sinks[kr] + 2)  # + the rollup's PFMERGE scratch slot
        if args.shard:  # verify() runs as one rank above this shard's slots
            self.sinks = [self.sinks[kr]]
            self.km_verify = _ShardView(self.km.slots_end(kr))
        else:
            self.km_verify = self.km
        self.variant = variant = engine.variant(0)
        self.lds_k1 = lds_k1 = variant == 1
        self.persistent = bool(args.persistent if args.persistent >= 0 else lds_k1) and not args.exchange
        if lds_k1:
            engine.set_option("k1_persistent", 1 if self.persistent else 0)
        streams_n = 1 if self.persistent else (args.streams or (16 if lds_k1 else 1))
        self.use_graph = 0 if self.persistent else (args.graph if args.graph >= 0 else (1 if lds_k1 else 0))
        k1_grid = args.k1_grid
        if k1_grid < 0:
            cus = torch.cuda.get_device_properties(local).multi_processor_count
            k1_grid = cus // 2 if (lds_k1 and streams_n > 1) else 0
        if k1_grid:
            engine.set_option("k1_grid", k1_grid)
        self.nb = nb = max(1, min(args.max_batches, args.steps + args.warmup))
        self.batches = [engine.swipe_batch(p, (rank * nb + j) * n, n) for j in range(nb)]
        self.out = DeviceBuffer(engine.ctx, n)  # BF.EXISTS answers (the reference stores is_valid)
        self.probes, self.nvalid = engine.swipes_stats(0, self.batches[0])
        self.width = synthetic.id_width(w)
        self.fixed = args.layout == "fixed"
        self.streams = [stream] + [torch.cuda.Stream() for _ in range(max(0, streams_n - 1))]
        self.ex, self.xviews = None, []
        if args.exchange:
            from rtsas_amd.distributed import SwipeExchange, engine_k1

            def tview(ptr, shape, typestr):  # zero-copy torch view of a library buffer
                class _V:
                    __cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False),
                                                "version": 3, "strides": None}
                return torch.as_tensor(_V(), device=dev)
            self.ex = SwipeExchange(rank, world, engine_k1(engine), self.km, engine=engine, sink_slots=self.sinks,
                                    overlap=args.exchange != 2)
            # (the ids' view keeps the batch buffer's padding in its storage:
            # K1 may read past the last id)
            self.xviews = [(tview(b.bytes.ptr, (n * self.width + 64,), "|u1")[:n * self.width].view(n, self.width),
                            tview(b.slot.ptr, (n,), "<i4")) for b in self.batches]

    # ---- steps
    def step(self, j):
        e = self.engine
        if self.ex is not None:
            # host-free exchange: equal splits of a capacity, settled at the end
            self.ex.swipes_async(*self.xviews[j % self.nb])
            return
        if len(self.streams) > 1:
            e.set_stream(self.streams[j % len(self.streams)].cuda_stream)
        if self.fixed:
            e.swipes_fixed_async(0, self.batches[j % self.nb], self.out)
        else:
            e.swipes_async(0, self.batches[j % self.nb], self.out)

    def warm(self):
        a, e = self.args, self.engine
        if self.persistent:
            # the timed call's batch descriptors (device pointers of the resident
            # batches), built once like the batches themselves
            self.many = e.many_args([self.batches[(a.warmup + j) % self.nb] for j in range(a.steps)],
                                    [self.out] * a.steps, fixed=self.fixed)
        if self.persistent:  # the same call shape as the timed region (loads the kernel)
            e.swipes_many_async(0, [self.batches[j % self.nb] for j in range(max(1, a.warmup))],
                                [self.out] * max(1, a.warmup), fixed=self.fixed)
        else:
            for j in range(a.warmup):
                self.step(j)
        e.set_stream(self.stream.cuda_stream)
        self.torch.cuda.synchronize()
        self.finish()
        e.check_errors()

    def finish(self):
        """The end of a run of steps: the exchange's settle (capacity
        overflows re-run with exact splits; a collective)."""
        if self.ex is not None:
            self.redone = getattr(self, "redone", 0) + self.ex.settle()

    def enqueue_steps(self, graph):
        a, e, torch = self.args, self.engine, self.torch
        if graph is not None:
            graph.launch()
        elif self.persistent:
            e.swipes_many_async(0, None, prepared=self.many)
        else:
            for s_ in self.streams[1:]:
                s_.wait_stream(self.stream)
            for j in range(a.steps):
                self.step(a.warmup + j)
            if self.ex is not None:
                # the pipelined exchange's last return half, and the timed
                # stream waits for its streams (inside the timed region)
                self.ex.flush()
            e.set_stream(self.stream.cuda_stream)
            for s_ in self.streams[1:]:
                self.stream.wait_stream(s_)

    def capture(self):
        a, e = self.args, self.engine
        if not self.use_graph:
            return None
        if len(self.streams) == 1:
            return e.capture(lambda: [self.step(a.warmup + j) for j in range(a.steps)])
        e.swipes_many_async(0, [], branches=len(self.streams))  # side streams, before capture
        self.torch.cuda.synchronize()
        return e.capture(lambda: e.swipes_many_async(
            0, [self.batches[(a.warmup + j) % self.nb] for j in range(a.steps)],
            [self.out] * a.steps, branches=len(self.streams), fixed=self.fixed))

    def timed(self, barrier=True):
        """Warm-up, then the K timed steps (no instrumentation)."""
        a, torch, dist = self.args, self.torch, self.dist
        self.warm()
        graph = self.capture()
        self.engine.set_option("pass_timing", 0)
        if barrier and self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(self.stream)
        self.enqueue_steps(graph)
        e1.record(self.stream)
        host_enqueue = time.perf_counter() - t0
        torch.cuda.synchronize()
        self.finish()
        if barrier and self.world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        self.engine.check_errors()  # an out-of-range slot in any timed step raises here
        self.graph = graph
        return elapsed, e0.elapsed_time(e1) / a.steps, host_enqueue

    def replay_instrumented(self):
        """The same warm-up + steps from a zeroed slab, every K1 kernel of the
        K steps bracketed by HIP events on its own stream: per-kernel times
        of the same work the timed region did.  A graph replays instead as a
        whole (its launch time / steps)."""
        a, e, torch = self.args, self.engine, self.torch
        if self.graph is not None:
            return None
        self.zero_slab()
        self.warm()
        e.set_option("pass_timing", 1)
        e.pass_times(reset=True)
        self.enqueue_steps(None)
        torch.cuda.synchronize()
        self.finish()
        e.set_option("pass_timing", 0)
        e.check_errors()
        return e.pass_times(reset=True)

    def zero_slab(self):
        p, nb = C.c_void_p(), C.c_uint64()
        self.engine.ctx.call("ske_hll_slab", C.byref(p), C.byref(nb))
        nbytes = self.nslots * 16384
        assert nbytes <= nb.value

        class _V:
            __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (p.value, False),
                                        "version": 3, "strides": None}
        self.torch.cuda.synchronize()
        self.torch.as_tensor(_V(), device=self.dev).zero_()
        self.torch.cuda.synchronize()

    def roofline(self, pt, step_ms):
        """§3's roofline on the kernel that takes the most time."""
        a, n = self.args, self.n
        cus = self.torch.cuda.get_device_properties(self.dev).multi_processor_count
        seg = bool(pt) and len(pt) > 5 and pt[5][1] > 0
        # per launch of the per-sub-batch kernels: one sub-batch (bench batches
        # are cut into even sub-batches of at most part_sub_default swipes)
        geom = chain_geometry(self.engine)
        nsub = -(-n // (a.part_sub or part_sub_default(geom)))
        alg = pass_bytes(n / nsub, self.nvalid / nsub, self.probes / nsub, self.width, self.fixed,
                         geom, lds_k1=self.lds_k1,
                         slab_bytes=(self.nslots if seg else self.nslots + VERIFY_KEYS) * 16384, cus=cus,
                         seg=seg, nsub=nsub)
        passes = {}
        for i, (ms, cnt) in enumerate((pt or [])[:K1_PASSES]):
            if cnt:
                mean = ms / cnt
                name = PASS_NAMES[i]
                # a persistent launch covers several steps and stages the filter once
                ab = (alg[name] * (a.steps / cnt if (self.persistent and name == "k1") else 1)
                      + (alg["k1_stage"] if name == "k1" else 0))
                passes[name] = {"ms": mean, "launches": cnt, "alg_bytes": ab,
                                "GBps": ab / (mean * 1e-3) / 1e9}
        if passes:
            # the kernel that takes the most time per step (a per-sub-batch
            # kernel launches nsub times per step, the window pass once)
            dom = max(passes, key=lambda k: passes[k]["ms"] * passes[k]["launches"])
            kern_ms, dom_bytes = passes[dom]["ms"], passes[dom]["alg_bytes"]
        else:  # graph replay: the launch time is the timed region's events / steps
            dom, kern_ms, dom_bytes = "k1", step_ms, alg["k1"] + alg["k1_stage"]
        achieved = dom_bytes / (kern_ms * 1e-3) / 1e9
        # HBM-side bytes per launch of that kernel from the committed rocprofv3
        # PMC passes of this workload (FETCH_SIZE + WRITE_SIZE, separate passes,
        # FETCH corrected for 16-B-per-lane streams where the summary says so)
        pmc, pmc_src = load_pmc(self.pmc_tag(seg), dom)
        traffic = None
        if pmc is not None and passes and dom != "k1":
            # a summary taken over launches of another size says nothing of these
            # (summaries before round 5's 2^25 sub-batches covered 2^24 swipes)
            per = n if dom == "k_seg_e" else n / nsub
            if abs(pmc.get("swipes_per_launch", 1 << 24) - per) > 0.01 * per:
                pmc, pmc_src = None, None
        if pmc is not None:
            # request-size-calibrated bytes where the summary has them (round 4:
            # every read request by its size, tools/fetchcal.hip), else FETCH+WRITE
            traffic = pmc.get("hbm_bytes_calibrated",
                              pmc.get("hbm_bytes_corrected", pmc.get("hbm_bytes_per_dispatch")))
            if traffic is not None and self.persistent and dom == "k1":
                # per launch of this run (one persistent launch per 48 steps
                # when the timed steps were not replayed per pass)
                launches = passes["k1"]["launches"] if "k1" in passes else -(-a.steps // 48)
                traffic *= a.steps / launches / pmc.get("steps_per_dispatch", a.steps)
        r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": achieved / HBM_PEAK_GBS,
             # also against the measured streaming rate
             "peak_measured": HBM_MEASURED_GBS, "frac_measured_peak": achieved / HBM_MEASURED_GBS,
             "traffic": traffic, "traffic_source": pmc_src, "pfadd_form": "segmented" if seg else "cas",
             "kernel": dom, "kernel_ms": kern_ms, "alg_bytes_per_launch": dom_bytes,
             "kernel_times": "instrumented replay of the timed steps" if passes else "timed region events",
             "device_ms_per_step": step_ms, "probes_per_swipe": self.probes / n,
             "valid_frac": self.nvalid / n, "passes": passes}
        if dom.startswith("k_part"):
            # SURVEY §8(d)'s whole-path model prices every probe as a random
            # 64-B HBM sector; the partitioned K1 answers probes from LDS slices
            whole = alg["k1"] * nsub
            r["whole_path_model"] = {
                "what": "SURVEY §8(d) bytes for the whole path (every probe a random 64-B sector): not an HBM "
                        "roofline for the partitioned K1, whose probes are served from LDS-resident filter "
                        "slices after a radix partition; its rooflines are the per-pass algorithmic bytes "
                        "(passes[*].alg_bytes), the dominant pass's taken above",
                "bytes_per_step": whole, "would_need_GBps": whole / (step_ms * 1e-3) / 1e9,
                "of_peak": whole / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        if dom == "k_part_c" and not seg:
            sectors = self.nvalid / nsub / (kern_ms * 1e-3) / 1e9
            r["random_sector_bound"] = {
                "what": "one 64-B HBM sector per valid swipe's register, against the measured random "
                        "4-B read rate over a 1.6 GB table (tools/randbench.hip)",
                "achieved_Gsectors_per_s": sectors, "peak_Gsectors_per_s": RANDOM_SECTOR_GPS,
                "frac": sectors / RANDOM_SECTOR_GPS}
            if pmc and "TCC_EA0_ATOMIC_sum" in pmc.get("mean", {}):
                req = (self.nvalid / nsub + pmc["mean"]["TCC_EA0_ATOMIC_sum"]) / (kern_ms * 1e-3) / 1e9
                r["random_sector_bound"].update({
                    "what": "random 64-B requests into the 1.6 GB register slab per second: one "
                            "pre-check load per valid swipe plus one memory-side CAS per raise "
                            "(TCC_EA0_ATOMIC_sum, PMC per dispatch), against the measured random 4-B "
                            "read rate over a 1.6 GB table (tools/randbench.hip)",
                    "achieved_Gsectors_per_s": req, "frac": req / RANDOM_SECTOR_GPS,
                    "loads_only_frac": sectors / RANDOM_SECTOR_GPS})
                cas = pmc["mean"]["TCC_EA0_ATOMIC_sum"] / (kern_ms * 1e-3) / 1e9
                r["binding"] = {
                    "counter": "TCC_EA0_ATOMIC_sum",
                    "what": "register CASes (memory-side device atomics, PMC per dispatch) / this run's "
                            "kernel time, against the measured rate of the same load + raising CAS "
                            "over a 1.6 GB table (tools/casbench.hip, profiles/r02_casbench.json)",
                    "atomics_per_dispatch": pmc["mean"]["TCC_EA0_ATOMIC_sum"],
                    "achieved_G_per_s": cas, "peak_G_per_s": RANDOM_CAS_GPS, "frac": cas / RANDOM_CAS_GPS}
        if dom == "k1" and pmc and "SQ_INSTS_VALU" in pmc.get("mean", {}):
            m = pmc["mean"]
            r["binding"] = {
                "counter": "SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_VALU",
                "what": "the LDS K1 is issue/latency bound, not HBM bound: per wave, the share of its "
                        "cycles waiting in s_waitcnt and issuing VALU (PMC of this workload's dispatch)",
                "wait_frac": m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"],
                "valu_frac": m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"],
                "valu_wave_insts_per_64_swipes":
                    m["SQ_INSTS_VALU"] / max(1.0, pmc.get("swipes_per_dispatch", 0) / 64),
                "lds_bank_conflict_rate": pmc.get("lds_bank_conflict_rate")}
        return r

    def pmc_tag(self, seg):
        """The name of this workload's committed PMC summaries
        (profiles/<round>_pmc_<tag>_<kernel>.json): the config, then the
        simulated shard, a non-default batch and the segmented PFADD."""
        a, tag = self.args, self.cfg
        if a.shard:
            tag += "_shard%d" % self.kw
        if a.batch and a.batch != BENCH_STEP.get(self.cfg, self.w.step_swipes):
            tag += "_b%dm" % (a.batch >> 20)
        return tag + ("_seg" if seg else "")

    def config(self):
        a, w = self.args, self.w
        shard = ({"shard_of": self.kw, "shard_rank": self.kr,
                  "what": "one rank's share of the %d-GPU job, run alone on this GPU" % self.kw}
                 if a.shard else {})
        return {"workload": w.name, **shard, "swipes_per_step": self.n, "students": w.n_members,
                "hll_keys_total": self.w_all.n_keys, "hll_keys_this_gpu": w.n_keys,
                "key_ownership": ("MurmurHash64A(key name, 0) mod world (distributed.KeyMap)" if a.ownership == "hash"
                                  else "mass-balanced: MurmurHash64A(key name, 0) mod 256 x world virtual buckets, "
                                       "assigned by greedy key mass (distributed.balanced_owners)"),
                "invalid_frac": w.invalid_frac,
                "bloom": {"error": w.bf_error, "capacity": w.bf_capacity},
                "id_bytes": self.width, "parallelism": f"dp{self.world} (key-sharded, Bloom replicated)",
                "k1_variant": {0: "global-bloom", 1: "lds-bloom", 2: "xcd-regions",
                               3: "partitioned"}[self.variant],
                "layout": a.layout, "streams": len(self.streams),
                "input": ("unpartitioned: equal-split all_to_all to the key owners per step "
                          "(SwipeExchange.swipes_async; capacity overflows re-run at settle)"
                          if a.exchange else "routed to the key owners at ingest"),
                "launch": ("hip-graph" if self.graph is not None else
                           ("persistent (one K1 launch per 48 steps)" if self.lds_k1 else
                            "one many-batch call")
                           if self.persistent else "host"),
                "answers": "written (1 B per swipe)"}

    def free(self):
        if getattr(self, "graph", None) is not None:
            self.graph.free()
        for b in self.batches:
            b.free()
        self.out.free()


def secondary(args, cfg, local, dev, dist):
    """A second configuration on its own context in the same process (N = 1)."""
    sargs = parse(["--config", cfg, "--steps", str(args.steps), "--warmup", str(args.warmup)])
    r = Run(sargs, cfg, 1, 0, local, dev, dist)
    elapsed, step_ms, _ = r.timed(barrier=False)
    pt = r.replay_instrumented() if args.pass_replay else None
    roof = r.roofline(pt, step_ms)
    keep = {k: roof[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_source",
                                 "kernel", "kernel_ms", "kernel_times", "binding") if k in roof}
    out = {"metric": METRIC, "value": r.n * sargs.steps / elapsed, "unit": "swipes/s",
           "steps": sargs.steps, "warmup": sargs.warmup, "ms_per_step": elapsed * 1e3 / sargs.steps,
           "device_ms_per_step": step_ms, "config": r.config(), "roofline": keep}
    r.free()
    return out


def main():
    args = parse()
    cmd = launch_plan(args, sys.argv[1:], os.environ)
    if cmd is not None:
        # N ranks as child processes, started before this process touches the
        # GPU (no torch.cuda, no libsketch here); rank 0's JSON line goes
        # straight to our stdout; a failing rank fails the run
        import subprocess
        print("bench.py: launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
        sys.exit(subprocess.run(cmd).returncode)
    import numpy as np  # noqa: F401
    import torch
    import torch.distributed as dist

    import __graft_entry__ as ge
    ge.load_package()
    from rtsas_amd import synthetic

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one GPU per rank; the modulo only matters for a rehearsal of several
    # ranks on a one-GPU box (--dist-backend gloo), never on a full node
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    if args.sync_spin:
        # torch's own HIP runtime (same soname): spin-wait host synchronisation,
        # which the timed region's closing synchronize() pays once per call
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so.7")
        if hip.hipSetDevice(local) == 0:
            hip.hipSetDeviceFlags(1)  # hipDeviceScheduleSpin
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":  # RCCL
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    run = Run(args, args.config, world, rank, local, dev, dist)
    elapsed, step_ms, host_enqueue = run.timed()
    free_b, total_b = torch.cuda.mem_get_info(dev)
    mem_used = float(total_b - free_b)  # the device's (all ranks on it: the rank's own on a node)
    cdev = dev if args.dist_backend == "nccl" else "cpu"
    my_elapsed = elapsed
    total_swipes = run.n
    shares = {"mode": run.shares, "swipes_per_step": [run.n], "key_mass": [run.mass],
              "elapsed_s": [elapsed], "device_mem_used_GB": [mem_used / 1e9]}
    if world > 1:
        t = torch.tensor([elapsed, step_ms], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, step_ms = float(t[0]), float(t[1])
        # every rank's batch, key mass and wall time (the slowest bounds the job)
        g = torch.zeros(4 * world, dtype=torch.float64, device=cdev)
        g[4 * rank:4 * rank + 4] = torch.tensor([run.n, run.mass, my_elapsed, mem_used], dtype=torch.float64)
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        g = g.view(world, 4).cpu().tolist()
        total_swipes = int(sum(r[0] for r in g))
        shares = {"mode": run.shares, "swipes_per_step": [int(r[0]) for r in g],
                  "key_mass": [r[1] for r in g], "elapsed_s": [r[2] for r in g],
                  "device_mem_used_GB": [r[3] / 1e9 for r in g],
                  "device_mem_note": "hipMemGetInfo used bytes of each rank's device after timing (ranks "
                                     "sharing a GPU in a rehearsal see their sum)"}
    # each rank's bytes over the inter-GPU links per step: none when input is
    # routed to the key owners at ingest; with --exchange, the capacity
    # layout's rows to every peer (id + local slot out, the answer back)
    if run.ex is not None and world > 1:
        cap = int(run.ex.stats.get("cap_rows_per_peer", 0))
        per_rank = cap * (world - 1) * (run.width + 4 + 1)
        shares["exchange_bytes_per_step"] = [per_rank] * world
        shares["exchange_what"] = ("rows to every peer (cap_rows_per_peer x (world - 1)) x (id %d B + slot 4 B "
                                   "out, answer 1 B back), per rank and step" % run.width)
    else:
        shares["exchange_bytes_per_step"] = [0] * world
        shares["exchange_what"] = "input routed to the key owners at ingest: no data-path exchange"
    mean_n = total_swipes / world
    shares.update({"rank_share_max": max(shares["swipes_per_step"]) / mean_n,
                   "rank_share_min": min(shares["swipes_per_step"]) / mean_n,
                   "slowest_rank": int(max(range(world), key=lambda r: shares["elapsed_s"][r]))})
    pt = run.replay_instrumented() if args.pass_replay else None
    pt_rank = rank
    if world > 1 and pt is not None:
        # the per-pass times of the slowest rank (the one that bounds the
        # job's time), every rank's gathered
        k = len(pt)
        t = torch.zeros(world * 2 * k, dtype=torch.float64, device=cdev)
        t[rank * 2 * k:(rank + 1) * 2 * k] = torch.tensor([x for ms, c in pt for x in (ms, c)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        allp = t.view(world, k, 2).cpu().tolist()
        pt_rank = shares["slowest_rank"]
        pt = [(float(ms), int(c)) for ms, c in allp[pt_rank]]
        shares["pass_ms_per_rank"] = [[ms / c if c else 0.0 for ms, c in r] for r in allp]

    ms_per_step = elapsed * 1e3 / args.steps
    value = total_swipes * args.steps / elapsed
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
        "data": "synthetic (device counter-based generator, seed %d)" % run.w.seed,
        "config": run.config(),
        "roofline": {**run.roofline(pt, step_ms), "passes_of_rank": pt_rank},
        "preload_s": run.preload_s,
        "host_enqueue_us_per_step": host_enqueue * 1e6 / args.steps,
        "rank_shares": shares,
    }
    line["config"]["swipes_per_step_all_ranks"] = total_swipes
    if args.stream_1b and not run.lds_k1 and not run.persistent and run.graph is None and not args.shard:
        line["stream_1b"] = checked(stream_1b, run, total_swipes, pt)
    if run.ex is not None:
        # cap_rows_per_peer / slack_used: what the timed steps were enqueued
        # with; slack_next: what settle() adapted it to for later batches
        line["exchange"] = {**run.ex.stats, "slack_next": run.ex.slack, "pipelined": run.ex.overlap}
    if (args.rollup if args.rollup >= 0 else args.config == "c5") and not args.shard and run.w_all.zipf_lectures:
        line["rollup"] = checked(rollup_bench, run, dist)
    if world == 1 and args.host_fed and not run.lds_k1:
        line["host_fed"] = checked(host_fed, run.engine, run.batches[0])
    want_cpu = rank == 0 and world == 1 and not args.no_cpu and args.cpu_seconds > 0
    if not args.no_check or want_cpu:
        orc = ge.load_oracle()
        chain = oracle_chain(run.engine, orc, run.w, run.p)
        if not args.no_check:
            chk = checked(verify, run.engine, orc, chain, run.w, run.km_verify, rank, world, dist, dev,
                          bool(args.exchange), run.sinks)
            if world > 1 and not args.exchange and getattr(verify, "last_map", None) is not None:
                # the unpartitioned-input path too (SwipeExchange: alltoallv over
                # RCCL at N > 1) on a third key universe, then the same queries
                x = checked(verify, run.engine, orc, chain, run.w, run.km, rank, world, dist, dev, True,
                            run.sinks, prefix="VERIFYX", under=verify.last_map)
                chk = {**chk, "ok": chk["ok"] and x["ok"], "exchange": x}
            line["check"] = chk
        if want_cpu:
            line["cpu_baseline"] = cpu_baseline(orc, chain, run.w, run.batches[0], args.cpu_seconds,
                                                lambda s: run.names[int(run.km.keys_of(run.kr)[s])])
    run.free()
    sec = args.secondary
    if sec == "auto":
        sec = "c2" if args.config == "c3" else "none"
    if world == 1 and sec != "none" and sec != args.config:
        line["secondary"] = secondary(args, sec, local, dev, dist)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
