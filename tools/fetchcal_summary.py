"""Per-kind FETCH_SIZE calibration from tools/fetchcal's rocprofv3 passes.

usage: python tools/fetchcal_summary.py gpurun_out/fetchcal

fetchcal launches each kernel 6 times, in order: k_stream16 (stream16),
k_strided4 (line4, then sector4), k_runs (runs, then runs_al).  For every kind
the counters are averaged over its 6 dispatches and set against the distinct
128-B lines the kind touches (times.json):
  fetch_per_line_B  = FETCH_SIZE (KB) * 1024 / lines   (128 if FETCH counted whole lines)
  factor            = 128 / fetch_per_line_B           (multiply FETCH_SIZE by it to get line bytes)
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import sys

KINDS = {"k_stream16": ["stream16"], "k_strided4": ["line4", "sector4"], "k_runs": ["runs", "runs_al"],
         "k_wstream16": ["wstream16"], "k_wbytes": ["wbytes"], "k_wstrided4": ["wline4"]}


def read_bytes(m: dict) -> float:
    """Memory-side read bytes from the TCC/EA request counters by size: 128-B
    requests at 128, 64-B at 64, 32-B at 32 (TCC_EA0_RDREQ counts them all)."""
    r128, r64 = m["TCC_EA0_RDREQ_128B_sum"], m["TCC_EA0_RDREQ_64B_sum"]
    r32 = m.get("TCC_EA0_RDREQ_32B_sum", 0.0)
    return 128 * r128 + 64 * r64 + 32 * r32


def main(root: str) -> dict:
    times = json.load(open(os.path.join(root, "times.json")))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        rows = collections.defaultdict(dict)
        order = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            name = next((k for k in KINDS if k in r["Kernel_Name"]), None)
            if name is None:
                continue
            d = int(r["Dispatch_Id"])
            if d not in rows[name]:
                order[name].append(d)
                rows[name][d] = {}
            rows[name][d][r["Counter_Name"]] = float(r["Counter_Value"])
        for name, kinds in KINDS.items():
            ds = sorted(order[name])
            for i, kind in enumerate(kinds):
                for d in ds[6 * i:6 * i + 6]:
                    for c, v in rows[name][d].items():
                        per[kind][c].append(v)
    out = {}
    for kind, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        t = times[kind]
        lines = t["lines"]
        e = {"ms": t["ms"], "lines": lines, "mean": m}
        if "FETCH_SIZE" in m:
            fpl = m["FETCH_SIZE"] * 1024 / lines
            e.update({"fetch_per_line_B": fpl, "factor": 128.0 / fpl if fpl else None})
        for c in ("TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
                  "TCC_EA0_RDREQ_128B_sum", "TCC_REQ_sum"):
            if c in m:
                e[c.replace("_sum", "") + "_per_line"] = m[c] / lines
        if "TCC_EA0_RDREQ_128B_sum" in m and "TCC_EA0_RDREQ_64B_sum" in m:
            # bytes by request size
            e["read_bytes_by_size"] = read_bytes(m)
            e["read_bytes_per_line"] = e["read_bytes_by_size"] / lines
        if "WRITE_SIZE" in m and "bytes" in t:
            # WRITE_SIZE (KB) against the bytes the kernel stores
            e["write_size_B"] = m["WRITE_SIZE"] * 1024
            e["write_size_per_stored_byte"] = m["WRITE_SIZE"] * 1024 / t["bytes"]
        for c in ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "TCC_WRITE_SECTORS_sum"):
            if c in m:
                e[c.replace("_sum", "") + "_per_line"] = m[c] / lines
        e["line_GBps"] = lines * 128 / (t["ms"] * 1e-3) / 1e9
        if "record_bytes" in t:
            e["record_bytes"] = t["record_bytes"]
            e["lines_per_record_byte"] = lines * 128 / t["record_bytes"]
        out[kind] = e
    return out


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1]), indent=1))
