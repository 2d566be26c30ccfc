"""Phase timeline of the short-id LDS K1 (sketch_k1.hip) on C2, from the
stamped diagnostic build (tools/stamps/libsketch_stamps.so, -DSKE_STAMPS).

Stamps (s_memtime, shader cycles; lane 0 of every wave):
  0 entry  1 first tile's loads + LDS-DMA issued  2 first tile hashed
  3 after the staging barrier  then per pipelined iteration i (i = 0, 1):
  4+3i probes done  5+3i registers / answers committed  6+3i next tile hashed
  15 exit
Prints, relative to the earliest entry on the same XCD (s_memtime counts per
XCD), the median / p90 / max over waves of every stamp, in microseconds at the
nominal 2.4 GHz.
usage: python tools/stamps/run_k1_stamps.py [batch]
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
eng = SketchEngine(0)
lib = eng.ctx.lib
lib.ske_diag_set_k1_stamp_buffer.argtypes = [C.c_void_p, C.c_void_p]
w = synthetic.WORKLOADS["c2"]
eng.reserve(0, w.bf_error, w.bf_capacity)
p = eng.gen_params(w)
eng.preload(0, p, w.n_members)
eng.hll_reserve(w.n_keys)
batches = [eng.swipe_batch(p, j * n, n) for j in range(12)]
nblocks, nwaves = 256, 16
N = nblocks * nwaves * 16
buf = DeviceBuffer(eng.ctx, N * 8)
lib.ske_diag_set_k1_stamp_buffer(eng.ctx.ptr, C.c_void_p(buf.ptr))
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
s = buf.to_host(np.uint64, N).reshape(nblocks * nwaves, 16).astype(np.int64)
ok = s[:, 0] > 0
xcd = (np.arange(nblocks * nwaves) // nwaves) % 8  # blocks are dealt round-robin over the XCDs
s, xcd = s[ok], xcd[ok]
# s_memtime counters are per XCD: times are taken relative to the earliest
# entry on the same XCD
t0 = np.array([s[xcd == x, 0].min() for x in range(8)])[xcd]
print(f"batch {n}: kernel {kern_us:.1f} us (events); {ok.sum()} waves stamped")
names = {0: "entry", 1: "loads+DMA issued", 2: "tile0 hashed", 3: "staging barrier",
         4: "it0 probes", 5: "it0 commit", 6: "it1 hashed", 7: "it1 probes", 8: "it1 commit",
         9: "it2 hashed", 10: "it2 probes", 11: "it2 commit", 15: "exit"}
for k, nm in names.items():
    col = s[:, k]
    m = col > 0
    if not m.any():
        continue
    us = (col[m] - t0[m]) / 2400.0
    print(f"  {k:2d} {nm:18s} median {np.median(us):7.2f} us   p90 {np.percentile(us, 90):7.2f}   "
          f"max {us.max():7.2f}   (n={m.sum()})")
