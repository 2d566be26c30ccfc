"""Benchmark of the fused validate-and-count hot path (K1: BF.EXISTS +
valid-gated PFADD) -- BASELINE.json's metric on its configs[1] (C2).

One step = one K1 launch over one resident batch of synthetic swipes (C2: 1M
swipes, 7-digit ids from a 100k-student population, 10 % invalid, 50
lecture-day HLL keys, Bloom RESERVE 0.01 / 100k preloaded).  Inputs are
generated on the GPU and resident in HBM before timing; each step consumes a
distinct batch of the stream.  The K timed steps are recorded once into a HIP
graph of sixteen independent branches (step j on branch j mod 16) and replayed;
K1 runs on one block per two CUs, so two consecutive steps run side by side,
each on half the chip, and one launch's fixed cost overlaps the other's
steady state (C2: 9.9 us per step against 13.2 us for one chain of
full-chip launches; --streams 1 gives that chain).  Overlapping launches have
no single duration and HIP events cannot time nodes inside a graph, so the
roofline's kernel duration comes from an untimed replay of the same K
launches as one chain, whose per-launch time equals rocprofv3's per-dispatch
average.
N>1: one process per GPU
(torchrun), each rank runs its own stream over its own key shard with the
Bloom replicated (no data-path collective; weak scaling).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import functools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "swipes/sec (fused BF.EXISTS+PFADD) at 1/2/4/8 GPUs; % of HBM peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--batch", type=int, default=0, help="swipes per step (default: config)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--tile", type=int, default=0, help="K1 swipes per thread in flight (1,2,4,8)")
    ap.add_argument("--variant", type=int, default=-1,
                    help="-1 auto, 0 global Bloom, 1 LDS Bloom, 2 XCD-partitioned Bloom")
    ap.add_argument("--max-batches", type=int, default=64)
    ap.add_argument("--ablate", type=int, default=0, help="diagnostic: K1 parts removed (bits)")
    ap.add_argument("--xr-u", type=int, default=0, help="XCD-partitioned K1: slice-pass tile")
    ap.add_argument("--xr-fu", type=int, default=0, help="XCD-partitioned K1: finish-pass tile")
    ap.add_argument("--part-sub", type=int, default=0,
                    help="partitioned K1: swipes per sub-batch of its three passes (0 = default)")
    ap.add_argument("--streams", type=int, default=16,
                    help="HIP streams the steps alternate over, so launch tails overlap "
                         "(with --graph 1: one graph of that many independent branches)")
    ap.add_argument("--k1-legacy", action="store_true",
                    help="diagnostic: the generic LDS K1 instead of the short-id kernel")
    ap.add_argument("--k1-grid", type=int, default=-1,
                    help="blocks of the short-id LDS K1 (0: one per CU; -1: one per CU with "
                         "--streams 1, else one per two CUs, so two consecutive steps run side "
                         "by side, each on half the CUs)")
    ap.add_argument("--graph", type=int, default=1,
                    help="1 = the K timed steps are recorded once into a HIP graph (one K1 "
                         "launch per step, each over its own resident batch, step j on branch "
                         "j mod --streams) and replayed; 0 = launched one by one from the host")
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


def cpu_baseline(engine, pkg, w, p, b0, seconds):
    """Oracle (C restatement of Redis/RedisBloom) running the processor loop
    attendance_processor.py:100-137 (BF.EXISTS then PFADD) on the same batch,
    repeated for ~`seconds`: half the time on all host threads
    (orc_process_swipes_mt, the reported value), half on 1 thread (SURVEY.md
    §8d item 2)."""
    import numpy as np
    import __graft_entry__ as ge
    orc = ge.load_oracle()
    mbatch = engine.members_batch(p, 0, w.n_members)
    mb, mo, _ = mbatch.to_host()
    mbatch.free()
    chain = orc.Chain(w.bf_capacity, w.bf_error)
    chain.madd_packed(mb, mo)
    buf, offs, slot = b0.to_host()
    slot = slot.astype(np.uint32)
    regs = np.zeros((int(slot.max()) + 1, 16384), np.uint8)
    n = len(offs) - 1

    def run(threads, budget):
        passes = 0
        t0 = time.perf_counter()
        while True:
            orc.process_swipes(chain, regs, slot, buf, offs, threads=threads)
            passes += 1
            if time.perf_counter() - t0 >= budget:
                break
        return passes, time.perf_counter() - t0

    nt = cpu_threads()
    p1, dt1 = run(1, seconds / 2)
    pm, dtm = run(nt, seconds / 2)
    return {"value": n * pm / dtm, "unit": "swipes/s", "cores": nt, "kind": "port",
            "sample": f"{pm} passes over the first {n}-swipe batch (C oracle, "
                      f"orc_process_swipes_mt, {nt} threads, {dtm:.1f}s)",
            "single_thread": {"value": n * p1 / dt1, "cores": 1,
                              "sample": f"{p1} passes, orc_process_swipes, {dt1:.1f}s"}}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import __graft_entry__ as ge
    pkg = ge.load_package()
    from rtsas_amd import synthetic
    from rtsas_amd.engine import SketchEngine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one GPU per rank; the modulo only matters for a rehearsal of several
    # ranks on a one-GPU box (--dist-backend gloo), never on a full node
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":  # RCCL
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)

    w_all = synthetic.WORKLOADS[args.config]
    w = synthetic.shard(w_all, world)
    n = args.batch or w.step_swipes
    engine = SketchEngine(local)
    # a dedicated (non-null) stream shared by libsketch and the timing events
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    engine.set_stream(stream.cuda_stream)
    if args.tile:
        engine.set_option("tile", args.tile)
    if args.variant >= 0:
        engine.set_option("variant", args.variant)
    if args.ablate:
        engine.set_option("ablate", args.ablate)
    if args.k1_grid < 0:
        cus = torch.cuda.get_device_properties(local).multi_processor_count
        args.k1_grid = cus // 2 if args.streams > 1 else 0
    if args.k1_grid:
        engine.set_option("k1_grid", args.k1_grid)
    if args.k1_legacy:
        engine.set_option("k1_legacy", 1)
    if args.xr_u:
        engine.set_option("xr_region_u", args.xr_u)
    if args.xr_fu:
        engine.set_option("xr_finish_u", args.xr_fu)
    if args.part_sub:
        engine.set_option("part_sub", args.part_sub)

    # Bloom preload (replicated on every rank), HLL key shard of this rank
    engine.reserve(0, w.bf_error, w.bf_capacity)
    p = engine.gen_params(w)
    t0 = time.perf_counter()
    engine.preload(0, p, w.n_members)
    preload_s = time.perf_counter() - t0
    engine.hll_reserve(w.n_keys)

    nb = max(1, min(args.max_batches, args.steps + args.warmup))
    batches = [engine.swipe_batch(p, (rank * nb + j) * n, n) for j in range(nb)]
    probes, nvalid = engine.swipes_stats(0, batches[0])
    width = len(str(w.id_hi - 1))

    fixed = args.layout == "fixed"
    streams = [stream] + [torch.cuda.Stream() for _ in range(max(0, args.streams - 1))]

    def step(j):
        if len(streams) > 1:
            engine.set_stream(streams[j % len(streams)].cuda_stream)
        if fixed:
            engine.swipes_fixed_async(0, batches[j % nb])
        else:
            engine.swipes_async(0, batches[j % nb])

    for j in range(args.warmup):
        step(j)
    torch.cuda.synchronize()
    graph = None
    if args.graph and len(streams) == 1:
        # the timed steps, recorded (not run) into one uploaded graph
        graph = engine.capture(lambda: [step(args.warmup + j) for j in range(args.steps)])
    elif args.graph and len(streams) > 1:
        one = engine.swipes_fixed_async if fixed else engine.swipes_async
        timed = [functools.partial(one, 0, batches[(args.warmup + j) % nb])
                 for j in range(args.steps)]
        # K1's average launch duration: HIP events cannot time event nodes
        # inside a graph, so the same K launches are first replayed (untimed)
        # as one chain on the kernel's stream, bracketed by an event pair
        engine.set_stream(stream.cuda_stream)
        cal = engine.capture(lambda: [fn() for fn in timed])
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        cal.launch()
        c1.record(stream)
        torch.cuda.synchronize()
        cal_ms = c0.elapsed_time(c1) / args.steps
        cal.free()
        # the timed graph: one native call, step j on branch j mod S
        # (ske_swipes_many_async forks its side streams from the context stream)
        engine.swipes_many_async(0, [], branches=len(streams))  # side streams, before capture
        torch.cuda.synchronize()
        graph = engine.capture(lambda: engine.swipes_many_async(
            0, [batches[(args.warmup + j) % nb] for j in range(args.steps)],
            branches=len(streams), fixed=fixed))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    # several streams: every launch is bracketed by its own event pair on the
    # stream it runs on, so the kernel's average duration is measured even
    # though consecutive launches overlap
    per = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)] if len(streams) > 1 and graph is None else []
    t0 = time.perf_counter()
    e0.record(stream)
    if graph is not None:
        graph.launch()
    else:
        for s_ in streams[1:]:
            s_.wait_stream(stream)
        for j in range(args.steps):
            if per:
                per[j][0].record(streams[(args.warmup + j) % len(streams)])
            step(args.warmup + j)
            if per:
                per[j][1].record(streams[(args.warmup + j) % len(streams)])
        for s_ in streams[1:]:
            stream.wait_stream(s_)
    e1.record(stream)
    host_enqueue = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    torch.cuda.synchronize()
    # average launch duration of K1: one stream -- HIP events around the K
    # back-to-back launches (includes the inter-kernel gaps, so an upper
    # bound); several streams -- the mean of the per-launch event pairs
    step_ms = e0.elapsed_time(e1) / args.steps
    kern_ms = sum(a.elapsed_time(b) for a, b in per) / len(per) if per else step_ms
    if graph is not None and len(streams) > 1:
        kern_ms = cal_ms
    if world > 1:
        t = torch.tensor([elapsed, kern_ms, step_ms], dtype=torch.float64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, step_ms = float(t[0]), float(t[1]), float(t[2])

    ms_per_step = elapsed * 1e3 / args.steps
    value = world * n * args.steps / elapsed
    # algorithmic bytes per launch: S_io per swipe (id bytes +
    # u32 offset + u32 slot + u8 answer), one 64-B sector per RedisBloom probe
    # (sequential count, measured), one 64-B sector read + write per PFADD
    s_io = width + (0 if fixed else 4) + 4 + 1
    # HBM-side bytes per K1 dispatch from the committed rocprofv3 PMC passes of
    # this same command (FETCH_SIZE + WRITE_SIZE, separate passes; see
    # profiles/README.md), or null when no summary exists for this workload
    traffic, traffic_src = None, None
    pmc_path = os.path.join(ROOT, "profiles", f"k1_pmc_{args.config}.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        traffic = pmc.get("hbm_bytes_per_dispatch")
        traffic_src = os.path.relpath(pmc_path, ROOT)
    alg_bytes = n * s_io + 64 * probes + 128 * nvalid
    variant = engine.variant(0)
    kernel_name = {0: "k_swipes", 1: "k_swipes" if args.k1_legacy else "k_swipes_lds",
                   2: "k_xr_hash+k_xr_region+k_xr_finish",
                   3: "k_part_a+k_part_b+k_part_c"}[variant]
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
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
                   "hll_keys_total": w_all.n_keys,
                   "hll_keys_per_gpu": w.n_keys, "invalid_frac": w.invalid_frac,
                   "bloom": {"error": w.bf_error, "capacity": w.bf_capacity},
                   "id_bytes": width, "parallelism": f"dp{world} (key-sharded, Bloom replicated)",
                   "k1_variant": {0: "global-bloom", 1: "lds-bloom", 2: "xcd-regions",
                                  3: "partitioned"}[variant],
                   "tile": args.tile or 2, "layout": args.layout, "streams": args.streams,
                   "k1_grid": args.k1_grid or "one block per CU",
                   "launch": "hip-graph" if graph is not None else "host"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": kernel_name, "kernel_ms": kern_ms,
                     "device_ms_per_step": step_ms,
                     "achieved_per_step": alg_bytes / (step_ms * 1e-3) / 1e9,
                     "alg_bytes_per_swipe": alg_bytes / n,
                     "probes_per_swipe": probes / n, "valid_frac": nvalid / n},
        "preload_s": preload_s,
        "host_enqueue_us_per_step": host_enqueue * 1e6 / args.steps,
    }
    if rank == 0 and not args.no_cpu and args.cpu_seconds > 0:
        line["cpu_baseline"] = cpu_baseline(engine, pkg, w, p, batches[0], args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if graph is not None:
        graph.free()
    for b in batches:
        b.free()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
