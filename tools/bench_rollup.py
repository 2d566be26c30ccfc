"""C5 campus-year rollup on one GPU (SURVEY.md §8d C5, rows a-9 .. a-11).

1. Preload the 10M-student Bloom (RESERVE 0.001 / 1e7, BF.MADD).
2. Ingest the 1B-swipe C5 stream into 365 days x 5000 lectures = 1.825M
   lecture-day HLL keys, generated on the device 16M swipes at a time.  The
   K1 time is summed from per-launch events; generation is not counted.
3. Time the rollup queries over the whole slab (30 GB of registers):
   - per-lecture unions: PFCOUNT of each lecture's 365 day keys (K2 with groups);
   - PFCOUNT of every lecture-day key (K2, one key per group);
   - the campus-wide PFMERGE of all 1.825M keys (two-level K3);
   - top / bottom-3 lectures (host, over the K2 counts).
Prints one JSON line with the times, the bytes read and the fraction of the
8 TB/s HBM peak.  usage: python tools/bench_rollup.py [--swipes N] [--lectures L]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--swipes", type=int, default=1_000_000_000)
    ap.add_argument("--lectures", type=int, default=5000)
    ap.add_argument("--days", type=int, default=365)
    ap.add_argument("--batch", type=int, default=16_000_000)
    args = ap.parse_args()
    ge.load_package()
    import torch
    from rtsas_amd import synthetic
    from rtsas_amd.engine import DeviceBuffer, SketchEngine
    from rtsas_amd.processor import rank_top_bottom

    w0 = synthetic.WORKLOADS["c5"]
    w = synthetic.Workload(**{**w0.__dict__, "zipf_lectures": args.lectures, "zipf_days": args.days,
                              "n_keys": args.lectures * args.days})
    eng = SketchEngine(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    t = time.perf_counter()
    eng.reserve(0, w.bf_error, w.bf_capacity)
    p = eng.gen_params(w)
    eng.preload(0, p, w.n_members)
    preload_s = time.perf_counter() - t
    eng.hll_reserve(w.n_keys)
    width = eng.ctx.lib.ske_gen_id_width(C.byref(p))

    # ---- ingest: 1B swipes, 16M per K1 launch
    from rtsas_amd.engine import DeviceBatch
    bufs = [DeviceBatch(eng.ctx, args.batch, width) for _ in range(2)]
    k1_ms, done, j = 0.0, 0, 0
    t = time.perf_counter()
    while done < args.swipes:
        n = min(args.batch, args.swipes - done)
        b = bufs[j % 2]
        eng.ctx.call("ske_gen_swipes", C.byref(p), done, n, C.c_void_p(b.bytes.ptr),
                     C.c_void_p(b.offs.ptr), C.c_void_p(b.slot.ptr))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.ctx.call("ske_swipes_async", 0, C.c_void_p(b.slot.ptr), C.c_void_p(b.bytes.ptr),
                     C.c_void_p(b.offs.ptr), n, None)
        e1.record(stream)
        e1.synchronize()
        k1_ms += e0.elapsed_time(e1)
        done += n
        j += 1
    ingest_s = time.perf_counter() - t

    nkeys = w.n_keys
    slab_bytes = nkeys * 16384

    def timed(fn, reps=3):
        """(best host wall s, best device s between events on the stream, out)"""
        fn()
        torch.cuda.synchronize()
        best, best_dev = 1e30, 1e30
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            out = fn()
            e1.record(stream)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
            best_dev = min(best_dev, e0.elapsed_time(e1) / 1e3)
        return best, best_dev, out

    # per-lecture unions: group g = lecture g's day keys g*days .. g*days+days
    slots = np.arange(nkeys, dtype=np.uint32)
    goffs = (np.arange(args.lectures + 1, dtype=np.uint32) * args.days).astype(np.uint32)
    out_g = np.zeros(args.lectures, np.uint64)
    d_slots, d_goffs = DeviceBuffer(eng.ctx, slots.nbytes), DeviceBuffer(eng.ctx, goffs.nbytes)
    d_slots.from_host(slots)
    d_goffs.from_host(goffs)
    d_out = DeviceBuffer(eng.ctx, nkeys * 8)

    def groups():  # host arrays in and out (the ABI copies them)
        eng.ctx.call("ske_hll_pfcount_groups", slots.ctypes.data_as(C.c_void_p),
                     goffs.ctypes.data_as(C.c_void_p), args.lectures,
                     out_g.ctypes.data_as(C.c_void_p), 0)
        return out_g

    def groups_dev():  # device-resident slots / offsets / counts: the kernel alone
        eng.ctx.call("ske_hll_pfcount_groups", C.c_void_p(d_slots.ptr), C.c_void_p(d_goffs.ptr),
                     args.lectures, C.c_void_p(d_out.ptr), 1)

    t_groups, _, lect_counts = timed(groups)
    _, k_groups, _ = timed(groups_dev)
    out_e = np.zeros(nkeys, np.uint64)

    def each():
        eng.ctx.call("ske_hll_pfcount_each", None, nkeys, out_e.ctypes.data_as(C.c_void_p), 0)
        return out_e

    def each_dev():
        eng.ctx.call("ske_hll_pfcount_each", None, nkeys, C.c_void_p(d_out.ptr), 1)

    t_each, _, key_counts = timed(each)
    _, k_each, _ = timed(each_dev)
    assert np.array_equal(d_out.to_host(np.uint64, nkeys), key_counts)
    eng.hll_reserve(nkeys + 1)
    campus = nkeys

    def merge():
        eng.ctx.call("ske_hll_clear", campus)
        eng.ctx.call("ske_hll_pfmerge", campus, slots.ctypes.data_as(C.c_void_p), nkeys)

    t_merge, k_merge, _ = timed(merge)
    campus_count = int(eng.pfcount_each(np.array([campus], np.uint32))[0])
    names = [f"LECT{i:05d}" for i in range(args.lectures)]
    t0 = time.perf_counter()
    head, tail = rank_top_bottom(lect_counts.astype(np.int64), names, 3)
    t_rank = time.perf_counter() - t0

    def gbs(sec):
        return slab_bytes / sec / 1e9

    line = {
        "workload": "c5-campus-year (1 GPU: the per-rank rollup; 8 GPUs shard the keys)",
        "keys": nkeys, "lectures": args.lectures, "days": args.days, "swipes": args.swipes,
        "slab_GB": slab_bytes / 1e9,
        "preload_s": preload_s,
        "ingest": {"k1_s": k1_ms / 1e3, "swipes_per_s": args.swipes / (k1_ms / 1e3),
                   "wall_s_incl_generation": ingest_s},
        "per_lecture_pfcount": {"s": t_groups, "kernel_s": k_groups, "GB_per_s": gbs(k_groups),
                                "hbm_frac": gbs(k_groups) / HBM_PEAK_GBS},
        "pfcount_each": {"s": t_each, "kernel_s": k_each, "keys_per_s": nkeys / k_each,
                         "GB_per_s": gbs(k_each), "hbm_frac": gbs(k_each) / HBM_PEAK_GBS},
        "campus_pfmerge": {"s": t_merge, "kernel_s": k_merge, "GB_per_s": gbs(k_merge),
                           "hbm_frac": gbs(k_merge) / HBM_PEAK_GBS, "pfcount": campus_count},
        "note": "s = host call incl. copies of the host arrays; kernel_s = device time between "
                "events with device-resident inputs / outputs; GB_per_s over kernel_s",
        "top3": {names[i]: int(lect_counts[i]) for i in head},
        "bottom3": {names[i]: int(lect_counts[i]) for i in tail},
        "rank_s": t_rank,
    }
    print(json.dumps(line), flush=True)
    for b in bufs + [d_slots, d_goffs, d_out]:
        b.free()


if __name__ == "__main__":
    main()
