"""Diagnostic: the partitioned K1 on a C3-geometry batch against the oracle;
prints where answers differ (tile, position in tile, false +/-).
usage: python tools/diag_part.py [n_swipes]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ge.load_package()
orc = ge.load_oracle()
from rtsas_amd import synthetic  # noqa: E402
from rtsas_amd.engine import DeviceBuffer, SketchEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 700_333
w = synthetic.WORKLOADS["c3"]
w = synthetic.Workload(**{**w.__dict__, "n_members": 300_000, "n_keys": 97, "zipf_lectures": 0, "zipf_days": 0,
                          "invalid_frac": 0.1})
eng = SketchEngine(0)
eng.reserve(0, w.bf_error, w.bf_capacity)
p = eng.gen_params(w, seed=4242)
eng.preload(0, p, w.n_members)
eng.hll_reserve(w.n_keys)
b = eng.swipe_batch(p, 7, n)
out = DeviceBuffer(eng.ctx, b.n)
eng.swipes(0, b, out)
chain = orc.Chain(w.bf_capacity, w.bf_error)
mb = eng.members_batch(p, 0, w.n_members).to_host()
chain.madd_packed(mb[0], mb[1])
regs = np.zeros((w.n_keys, 16384), np.uint8)
buf, offs, slot = b.to_host()
v, nvalid, _ = orc.process_swipes(chain, regs, slot.astype(np.uint32), buf, offs)
got = out.to_host(np.uint8, b.n)
bad = np.nonzero(got != v)[0]
print("n", n, "tiles", -(-n // 1024), "mismatches", bad.size, "false_pos", int(((got == 1) & (v == 0)).sum()),
      "false_neg", int(((got == 0) & (v == 1)).sum()))
if bad.size:
    t = bad // 1024
    ut, ct = np.unique(t, return_counts=True)
    print("tiles with mismatches", ut.size, "first", ut[:20].tolist(), "counts", ct[:20].tolist())
    print("tile % 8 (XCD group of pass A? no: groups are contiguous)", np.bincount(t % 8, minlength=8).tolist())
    ntiles = -(-n // 1024)
    g = (t * 8) // ntiles
    print("tile group (contiguous eighths)", np.bincount(g, minlength=8).tolist())
    pos = bad % 1024
    print("position in tile: <512", int((pos < 512).sum()), ">=512", int((pos >= 512).sum()))
    # index of the tile within its group -> which block / iteration of pass A
    t0 = (np.arange(8) * ntiles) // 8
    ig = t - t0[g]
    print("tile index within group: iteration (ig // 64)", np.bincount(ig // 64).tolist(), "parity", np.bincount((ig // 64) % 2).tolist())
print("registers equal", bool(np.array_equal(eng.registers_all(w.n_keys), regs)))
