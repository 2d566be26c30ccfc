"""Per-window timeline of the segmented PFADD's window pass (k_seg_e E1 / E2)
from the stamped diagnostic build (tools/stamps/libsketch_segstamps.so, the
library built with EXTRA=-DSKE_SEG_STAMPS).  Runs one bench batch to warm the
slab, then stamps the next batch's window pass: per window / queued slice,
s_memrealtime (100 MHz) at entry, after the run-table count, after the LDS
image (apply start), after the raises, at exit; its records, runs and block.
Prints phase percentiles, the busiest block's sum and the pass span.
usage: SKE_LIB=tools/stamps/libsketch_segstamps.py python tools/stamps/run_seg_stamps.py [bench args]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("SKE_LIB", os.path.join(ROOT, "tools", "stamps", "libsketch_segstamps.so"))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

ge.load_package()
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

args = bench.parse(["--steps", "1", "--warmup", "1", "--no-cpu", "--no-check", "--secondary", "none",
                    "--host-fed", "0"] + sys.argv[1:])
torch.cuda.set_device(0)
run = bench.Run(args, args.config, 1, 0, 0, torch.device("cuda", 0), dist)
eng = run.engine
lib = eng.ctx.lib
lib.ske_diag_set_seg_stamp_buffer.argtypes = [C.c_void_p, C.c_void_p]
buf = torch.zeros(1 << 21, dtype=torch.int64, device="cuda")
eng.swipes(0, run.batches[0], run.out)  # warm slab
torch.cuda.synchronize()
lib.ske_diag_set_seg_stamp_buffer(eng.ctx.ptr, C.c_void_p(buf.data_ptr()))
eng.swipes(0, run.batches[1 % run.nb], run.out)
torch.cuda.synchronize()
lib.ske_diag_set_seg_stamp_buffer(eng.ctx.ptr, None)
st = buf.view(-1, 8).cpu().numpy()
used = st[:, 4] > 0
idx = np.nonzero(used)[0]
st = st[used]
t0 = st[:, 0].min()
info = st[:, 5].astype(np.uint64)
nrec = (info & np.uint64(0xffffffff)).astype(np.int64)
npairs = ((info >> np.uint64(32)) & np.uint64(0x7fffffff)).astype(np.int64)
block = (st[:, 6] & 0xffffffff).astype(np.int64)
ph = np.diff(st[:, :5], axis=1) / 100.0  # us: count, image, apply, write
tot = (st[:, 4] - st[:, 0]) / 100.0
res = {"items": int(used.sum()), "span_us": float((st[:, 4].max() - t0) / 100.0)}
nwin_guess = int(idx.max()) + 1
for name, sel in (("all", np.ones(len(st), bool)),):
    q = lambda a: [float(np.percentile(a, p)) for p in (50, 90, 99, 100)]
    res[name] = {"count_us_p50_90_99_max": q(ph[:, 0]), "image_us": q(ph[:, 1]), "apply_us": q(ph[:, 2]),
                 "write_us": q(ph[:, 3]), "total_us": q(tot), "records": q(nrec), "runs": q(npairs)}
# split: items of E1 (index < nwin) vs E2, and by run count (hot buckets)
e2 = idx >= nwin_guess_e1 if False else None
hot = npairs > 1024
for name, sel in (("runs_le_1024", ~hot), ("runs_gt_1024", hot)):
    if sel.any():
        res[name] = {"items": int(sel.sum()), "sum_us": float(tot[sel].sum()),
                     "total_us_p50_90_max": [float(np.percentile(tot[sel], p)) for p in (50, 90, 100)],
                     "phases_mean_us": [float(x) for x in ph[sel].mean(axis=0)],
                     "records_mean": float(nrec[sel].mean())}
res["e1_end_us"] = float((st[idx < int(os.environ.get("NWIN", "1e12")), 4].max() - t0) / 100.0) if "NWIN" in os.environ else None
per_block = np.bincount(block, weights=tot)
res["busiest_block_sum_us"] = float(per_block.max())
res["mean_block_sum_us"] = float(per_block[per_block > 0].mean())
res["apply_us_per_1k_records_median"] = float(np.median(ph[:, 2] / np.maximum(1, nrec) * 1000))
big = np.argsort(-tot)[:8]
res["slowest"] = [{"item": int(idx[i]), "us": float(tot[i]), "phases": [float(x) for x in ph[i]],
                   "records": int(nrec[i]), "runs": int(npairs[i]), "block": int(block[i]),
                   "start_us": float((st[i, 0] - t0) / 100.0)} for i in big]
print(json.dumps(res))
