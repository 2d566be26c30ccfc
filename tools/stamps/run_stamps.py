"""Phase timeline of K1 (LDS variant, C2) from the stamped diagnostic build.

Stamps per wave and tile (s_memtime ticks, lane 0):
  0 kernel entry   1 tile start   2 id/slot loads issued (+ Bloom staged, tile 0)
  3 hashes + HLL pre-check issued   4 probes done   5 HLL CAS done
Prints median / p90 phase lengths in microseconds (100 MHz s_memrealtime is not
used; s_memtime runs at the shader clock, so ticks are converted with the
clock measured over the whole kernel: ticks(last stamp) / kernel wall time).
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
from rtsas_amd import _lib, synthetic  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "tools", "stamps", "libsketch_stamps.so")
from rtsas_amd.engine import DeviceBuffer, SketchEngine  # noqa: E402

import torch  # noqa: E402

eng = SketchEngine(0)
lib = eng.ctx.lib
lib.ske_diag_set_stamp_buffer.argtypes = [C.c_void_p, C.c_void_p]
w = synthetic.WORKLOADS["c2"]
tile = int(sys.argv[1]) if len(sys.argv) > 1 else 2
eng.set_option("tile", tile)
eng.reserve(0, w.bf_error, w.bf_capacity)
p = eng.gen_params(w)
eng.preload(0, p, w.n_members)
eng.hll_reserve(w.n_keys)
batches = [eng.swipe_batch(p, j * w.step_swipes, w.step_swipes) for j in range(12)]
nblocks, nwaves = 256, 16
buf = DeviceBuffer(eng.ctx, nblocks * nwaves * 2 * 8 * 8)
lib.ske_diag_set_stamp_buffer(eng.ctx.ptr, C.c_void_p(buf.ptr))
for j in range(11):
    eng.swipes(0, batches[j])
torch.cuda.synchronize()
s = buf.to_host(np.uint64, nblocks * nwaves * 2 * 8).reshape(nblocks, nwaves, 2, 8).astype(np.int64)
t0 = s[:, :, 0, 0][s[:, :, 0, 0] > 0].min()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
eng.swipes(0, batches[11])
ev[1].record()
torch.cuda.synchronize()
kern_us = ev[0].elapsed_time(ev[1]) * 1e3
s = buf.to_host(np.uint64, nblocks * nwaves * 2 * 8).reshape(nblocks, nwaves, 2, 8).astype(np.int64)
valid = s[:, :, 0, 0] > 0
start = s[:, :, 0, 0][valid].min()
last = s[valid].max()
ghz = (last - start) / (kern_us * 1e3)
print(f"tile={tile} kernel {kern_us:.1f} us (events), stamped span {(last - start) / ghz / 1e3:.1f} us "
      f"at {ghz:.2f} GHz-equivalent ticks")
names = {(0, 1): "entry->tile0", (1, 2): "loads+stage", (2, 3): "hash+precheck issue",
         (3, 4): "probes", (4, 5): "HLL wait+CAS"}
for t in range(2):
    for (a, b), nm in names.items():
        if t == 1 and a == 0:
            continue
        d = (s[:, :, t, b] - s[:, :, t, a])[valid & (s[:, :, t, b] > 0)] / ghz / 1e3
        if d.size:
            print(f"  tile{t} {nm:22s} median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f} us")
    if t == 0:
        d = (s[:, :, 1, 1] - s[:, :, 0, 5])[valid & (s[:, :, 1, 1] > 0)] / ghz / 1e3
        if d.size:
            print(f"  out writes+loop        median {np.median(d):6.2f} us")
ends = np.maximum(s[:, :, 0, 5], s[:, :, 1, 5])[valid]
print(f"  wave end (last stamp) rel. to first entry: median {np.median(ends - start) / ghz / 1e3:.2f} us, "
      f"max {(ends.max() - start) / ghz / 1e3:.2f} us; first entry spread "
      f"{(s[:, :, 0, 0][valid].max() - start) / ghz / 1e3:.2f} us")
