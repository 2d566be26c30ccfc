"""Where pass C's register atomics come from (C3, one GPU): a host simulation
of the bench's stream (the numpy restatement of the device generator,
tests/golden/gen_ref.py) through Redis' hllPatLen, step by step.

Per 16M-swipe step it reports, for the valid swipes:
  * updates            -- PFADDs reaching pass C (one pre-check load each)
  * raises_vs_start    -- updates whose rank exceeds the register's value at
                          the start of the step (what a pre-check load sees
                          when no other update of the step got there first:
                          ~ pass C's memory-side CASes, TCC_EA0_ATOMIC)
  * distinct_raised    -- distinct registers that rise in the step (the
                          floor of ANY scheme that writes each raised
                          register once per step, e.g. full dedup by sort)
  * distinct_lines     -- distinct 128-B register lines that rise (the
                          floor of line-owned PFADD, hll_mode 1)
split by lecture: the hottest lecture (Zipf rank 1: ~16 % of the stream,
its 100 day keys = 1.6 MB of registers), lectures 2-10, the rest.  This is
the evidence for DESIGN.md §3's pass C bound: what LDS-staging the hot keys
or deduplicating within a step could save.

usage: python tools/sim_raises.py [steps] [out.json]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def hll_idx_rank(ids: np.ndarray, width: int):
    """hllPatLen of decimal ids: (register, rank) -- MurmurHash64A seed 0xadc83b19."""
    from rtsas_amd.keyhash import _murmur_same_len
    digits = np.zeros((ids.size, width), np.uint8)
    x = ids.astype(np.uint64).copy()
    for d in range(width - 1, -1, -1):
        digits[:, d] = (x % np.uint64(10)).astype(np.uint8) + 48
        x //= np.uint64(10)
    h = _murmur_same_len(digits, 0xADC83B19)
    idx = (h & np.uint64(16383)).astype(np.int64)
    w = (h >> np.uint64(14)) | (np.uint64(1) << np.uint64(50))
    # rank = 1 + count of trailing zeros of w
    low = w & (~w + np.uint64(1))
    rank = np.log2(low.astype(np.float64)).astype(np.int64) + 1
    return idx, rank


def main():
    import __graft_entry__ as ge
    ge.load_package()
    from gen_ref import Gen
    from rtsas_amd import synthetic
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 25
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    w = synthetic.WORKLOADS["c3"]
    p = synthetic.gen_params(w)
    g = Gen(p)
    cdf = synthetic.key_cdf(w)
    n = w.step_swipes
    days = w.zipf_days
    regs = np.zeros(w.n_keys * 16384, np.uint8)
    rows = []
    for s in range(steps):
        t0 = time.time()
        start = s * n
        i = np.arange(start, start + n, dtype=np.uint64)
        from gen_ref import mix
        invalid = (mix(g.seed, i, 0) >> np.uint64(32)) < np.uint64(g.inv_thr)
        valid = ~invalid
        ids = g.member(mix(g.seed, i[valid], 1) % np.uint64(g.N))
        slot = g.swipe_slots(start, n, cdf)[valid].astype(np.int64)
        idx, rank = hll_idx_rank(ids, synthetic.id_width(w))
        flat = slot * 16384 + idx
        old = regs[flat]
        # exact no-op filters from summaries taken at the step's start: the
        # key's minimum register, and its 128-register line's minimum (an
        # update with rank <= the minimum cannot raise anything)
        kmin = regs.reshape(w.n_keys, 16384).min(axis=1)
        lmin = regs.reshape(w.n_keys * 128, 128).min(axis=1)
        skip_key = rank <= kmin[slot]
        skip_line = rank <= lmin[flat // 128]
        up = rank > old
        lect = slot // days
        cls = np.where(lect == 0, 0, np.where(lect < 10, 1, 2))
        # per register: the step's max rank
        order = np.argsort(flat, kind="stable")
        fs, rs = flat[order], rank[order]
        first = np.r_[True, fs[1:] != fs[:-1]]
        starts = np.nonzero(first)[0]
        mx = np.maximum.reduceat(rs, starts)
        keys = fs[starts]
        rose = mx > regs[keys]
        regs[keys[rose]] = mx[rose].astype(np.uint8)
        kcls = np.where(keys // 16384 // days == 0, 0, np.where(keys // 16384 // days < 10, 1, 2))
        lines = np.unique(keys[rose] // 128)
        lcls = np.where(lines * 128 // 16384 // days == 0, 0, np.where(lines * 128 // 16384 // days < 10, 1, 2))
        row = {"step": s, "updates": int(valid.sum()), "raises_vs_start": int(up.sum()),
               "skippable_key_min": int(skip_key.sum()), "skippable_line_min": int(skip_line.sum()),
               "distinct_raised": int(rose.sum()), "distinct_lines": int(lines.size),
               "by_class": {name: {"updates": int((cls == c).sum()), "raises_vs_start": int((up & (cls == c)).sum()),
                                   "distinct_raised": int((rose & (kcls == c)).sum()),
                                   "distinct_lines": int((lcls == c).sum())}
                            for c, name in enumerate(["lecture_1", "lectures_2_10", "rest"])},
               "seconds": round(time.time() - t0, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump({"workload": w.name, "step_swipes": n, "steps": rows}, f, indent=1)


if __name__ == "__main__":
    main()
