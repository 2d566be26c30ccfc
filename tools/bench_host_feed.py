"""PCIe-inclusive rate of the C3 step: the same 16M-swipe batch
as bench.py, but handed over in HOST memory through ske_swipes(...,
SKE_MEM_HOST): ids, offsets and key slots are staged host -> device by the
library, K1 runs, the answers come back device -> host, and the call returns
after its stream completed.  Timed for pageable numpy buffers and for pinned
(page-locked) torch buffers.  Never the bench's `value`: that one starts with
the batch resident in HBM.  usage: python tools/bench_host_feed.py [--reps R]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--config", default="c3")
    args = ap.parse_args()
    import torch
    ge.load_package()
    from rtsas_amd import synthetic
    from rtsas_amd._lib import SKE_MEM_HOST
    from rtsas_amd.engine import DeviceBuffer, SketchEngine

    w = synthetic.WORKLOADS[args.config]
    eng = SketchEngine(0)
    eng.reserve(0, w.bf_error, w.bf_capacity)
    p = eng.gen_params(w)
    eng.preload(0, p, w.n_members)
    eng.hll_reserve(w.n_keys + 64)
    n = w.step_swipes
    b = eng.swipe_batch(p, 0, n)
    buf, offs, slot = b.to_host()
    out_dev = DeviceBuffer(eng.ctx, n)
    eng.swipes(0, b, out_dev)  # the device-resident reference answers
    want = out_dev.to_host(np.uint8, n)

    def run(bbuf, boffs, bslot, bout, label):
        ptr = lambda a: C.c_void_p(a.ctypes.data if isinstance(a, np.ndarray) else a.data_ptr())
        eng.ctx.call("ske_swipes", 0, ptr(bslot), ptr(bbuf), ptr(boffs), n, ptr(bout), SKE_MEM_HOST)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            eng.ctx.call("ske_swipes", 0, ptr(bslot), ptr(bbuf), ptr(boffs), n, ptr(bout), SKE_MEM_HOST)
            ts.append(time.perf_counter() - t0)
        got = bout if isinstance(bout, np.ndarray) else bout.numpy()
        t = float(np.median(ts))
        return {"label": label, "ms_per_step": t * 1e3, "swipes_per_s": n / t,
                "host_bytes_per_step": int(bbuf.nbytes + boffs.nbytes + bslot.nbytes + n),
                "GB_per_s_host_link": (bbuf.nbytes + boffs.nbytes + bslot.nbytes + n) / t / 1e9,
                "answers_equal_device_resident": bool(np.array_equal(got, want))}

    res = [run(buf, offs, slot, np.zeros(n, np.uint8), "pageable numpy")]
    # fixed-width ids, answers 1 bit per swipe, chunked copy/compute pipeline
    width = int(offs[1] - offs[0])
    ids = np.ascontiguousarray(buf[:n * width].reshape(n, width))

    def run_bits(bids, bslot, bbits, label):
        ptr = lambda a: C.c_void_p(a.ctypes.data if isinstance(a, np.ndarray) else a.data_ptr())
        call = lambda: eng.ctx.call("ske_swipes_fixed_bits", 0, ptr(bslot), ptr(bids), width, n, ptr(bbits),
                                    SKE_MEM_HOST)
        call()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
        got = bbits if isinstance(bbits, np.ndarray) else bbits.numpy()
        t = float(np.median(ts))
        nbytes = int(n * width + bslot.nbytes + (n + 7) // 8)
        return {"label": label, "ms_per_step": t * 1e3, "swipes_per_s": n / t, "host_bytes_per_step": nbytes,
                "GB_per_s_host_link": nbytes / t / 1e9,
                "answers_equal_device_resident": bool(np.array_equal(
                    np.unpackbits(got, count=n, bitorder="little"), want))}
    res.append(run_bits(ids, slot, np.zeros((n + 7) // 8, np.uint8), "fixed width + bit answers, pageable numpy"))
    pid = torch.from_numpy(ids.reshape(-1)).pin_memory()
    pslot = torch.from_numpy(slot).pin_memory()
    pbits = torch.zeros((n + 7) // 8, dtype=torch.uint8).pin_memory()
    res.append(run_bits(pid, pslot, pbits, "fixed width + bit answers, pinned torch"))
    pb = torch.from_numpy(buf).pin_memory()
    po = torch.from_numpy(offs).pin_memory()
    ps = torch.from_numpy(slot).pin_memory()
    pout = torch.zeros(n, dtype=torch.uint8).pin_memory()
    res.append(run(pb, po, ps, pout, "pinned torch"))
    # the link alone: the same bytes pinned host -> device (torch), and back
    dev = [torch.empty(t.numel(), dtype=t.dtype, device="cuda") for t in (pb, po, ps)]
    dout = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        for d, h in zip(dev, (pb, po, ps)):
            d.copy_(h, non_blocking=True)
        pout.copy_(dout, non_blocking=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    res.append({"label": "link only (pinned, torch copies, no K1)", "ms_per_step": t * 1e3,
                "GB_per_s_host_link": (buf.nbytes + offs.nbytes + slot.nbytes + n) / t / 1e9})
    # host-side offset validation of the staging path alone
    t0 = time.perf_counter()
    ok = bool(np.all(offs[1:] >= offs[:-1]))
    res.append({"label": "numpy check of the offsets (host)", "ms": (time.perf_counter() - t0) * 1e3,
                "ok": ok})
    print(json.dumps({"workload": f"{args.config} one step ({n} swipes, host-resident batch)",
                      "results": res,
                      "note": "ske_swipes(..., SKE_MEM_HOST): H2D staging of ids/offsets/slots, K1, "
                              "D2H of the answers, synchronous; median of reps; PFADD repeats the "
                              "same batch (registers already raised after the first call)"}))


if __name__ == "__main__":
    main()
