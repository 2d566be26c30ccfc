"""Phase timeline of K1 (LDS variant, C2) from the stamped diagnostic build.

Stamps per wave and tile (s_memrealtime ticks at 100 MHz, lane 0):
  0 kernel entry   1 tile start   2 id/slot loads issued (+ Bloom staged, tile 0)
  3 hashes + HLL pre-check issued   4 probes done   5 HLL CAS done
Prints median / p90 phase lengths in microseconds.  The stamp buffer is zeroed
before the measured launch, which runs asynchronously on its own stream
between two events.
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
N = nblocks * nwaves * 2 * 8
buf = DeviceBuffer(eng.ctx, N * 8)
lib.ske_diag_set_stamp_buffer(eng.ctx.ptr, C.c_void_p(buf.ptr))
for j in range(10):
    eng.swipes_async(0, batches[j])
torch.cuda.synchronize()
buf.from_host(np.zeros(N, np.uint64))
stream = torch.cuda.Stream()
eng.set_stream(stream.cuda_stream)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(stream)
eng.swipes_async(0, batches[10])
ev[1].record(stream)
torch.cuda.synchronize()
kern_us = ev[0].elapsed_time(ev[1]) * 1e3
s = buf.to_host(np.uint64, N).reshape(nblocks, nwaves, 2, 8).astype(np.int64)
TICK_US = 0.01  # s_memrealtime: 100 MHz
valid = s[:, :, 0, 0] > 0
start = s[:, :, 0, 0][valid].min()
print(f"tile={tile} kernel {kern_us:.1f} us (events); {valid.sum()} waves stamped")
names = [(0, 1, "entry->tile0"), (1, 2, "loads(+stage)"), (2, 3, "hash+precheck issue"),
         (3, 4, "probes"), (4, 5, "HLL wait+CAS")]
for t in range(2):
    ok_t = valid & (s[:, :, t, 5] > 0)
    for a_, b_, nm in names:
        if t == 1 and a_ == 0:
            continue
        d = (s[:, :, t, b_] - s[:, :, t, a_])[ok_t] * TICK_US
        if d.size:
            print(f"  tile{t} {nm:22s} median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f} us  (n={d.size})")
    if t == 0:
        ok1 = valid & (s[:, :, 1, 1] > 0)
        d = (s[:, :, 1, 1] - s[:, :, 0, 5])[ok1] * TICK_US
        if d.size:
            print(f"  out writes+loop          median {np.median(d):6.2f} us")
entry = (s[:, :, 0, 0][valid] - start) * TICK_US
last = np.where(s[:, :, 1, 5] > 0, s[:, :, 1, 5], s[:, :, 0, 5])[valid]
print(f"  wave entry spread: median {np.median(entry):.2f} us, max {entry.max():.2f} us")
print(f"  wave end rel. first entry: median {np.median((last - start) * TICK_US):.2f} us, "
      f"max {(last.max() - start) * TICK_US:.2f} us")
