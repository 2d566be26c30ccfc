"""Per-block timeline of the partitioned K1's pass B (C3) from the stamped
diagnostic build (tools/ab/libsketch_stamps.so: tools/ab_variants.sh stamps
-DSKE_STAMPS).  Runs the bench's C3 workload for a few steps, stamps the last
step's pass B (s_memrealtime at 100 MHz, block entry / exit, the block's XCD)
and prints, per XCD, the blocks' start offsets and durations in microseconds:
a pass whose time is set by a slow XCD or by late-starting blocks shows here.
usage: python tools/stamps/run_pb_stamps.py [steps]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.load_package()
from rtsas_amd import _lib, synthetic  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "tools", "ab", "libsketch_stamps.so")
from rtsas_amd.engine import DeviceBuffer, SketchEngine  # noqa: E402

import torch  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
eng = SketchEngine(0)
lib = eng.ctx.lib
lib.ske_diag_set_pb_stamp_buffer.argtypes = [C.c_void_p, C.c_void_p]
w = synthetic.WORKLOADS["c3"]
eng.reserve(0, w.bf_error, w.bf_capacity)
wg = synthetic.Workload(**{**w.__dict__, "zipf_lectures": 0, "zipf_days": 0})  # keys do not matter to pass B
p = eng.gen_params(wg)
eng.preload(0, p, w.n_members)
eng.hll_reserve(w.n_keys)
assert eng.variant(0) == 3
n = w.step_swipes
batches = [eng.swipe_batch(p, j * n, n) for j in range(steps)]
out = DeviceBuffer(eng.ctx, n)
buf = torch.zeros(4096 * 4, dtype=torch.int64, device="cuda")
for j in range(steps):
    if j == steps - 1:
        torch.cuda.synchronize()
        buf.zero_()
        torch.cuda.synchronize()
        lib.ske_diag_set_pb_stamp_buffer(eng.ctx.ptr, C.c_void_p(buf.data_ptr()))
    eng.swipes(0, batches[j], out)
torch.cuda.synchronize()
lib.ske_diag_set_pb_stamp_buffer(eng.ctx.ptr, None)
st = buf.view(-1, 4).cpu().numpy()
used = st[:, 1] > 0
st = st[used]
t0 = st[:, 0].min()
start = (st[:, 0] - t0) / 100.0
dur = (st[:, 1] - st[:, 0]) / 100.0
end = (st[:, 1] - t0) / 100.0
xcc = st[:, 2] & 0xF
res = {"blocks": int(used.sum()), "pass_us": float(end.max()), "per_xcd": {}}
for x in sorted(set(xcc.tolist())):
    m = xcc == x
    res["per_xcd"][int(x)] = {"blocks": int(m.sum()), "start_max_us": round(float(start[m].max()), 2),
                              "dur_med_us": round(float(np.median(dur[m])), 2),
                              "dur_max_us": round(float(dur[m].max()), 2),
                              "end_max_us": round(float(end[m].max()), 2)}
print(json.dumps(res))
