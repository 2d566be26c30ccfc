"""Summarise rocprofv3 --pmc passes for one kernel into a JSON file.

usage: python tools/pmc_summary.py <pmc_root_dir> <kernel-substring> <out.json> [skip]

Each sub-directory of <pmc_root_dir> is one rocprofv3 pass
(<pass>/run_counter_collection.csv).  Per counter the value is averaged over
the dispatches of the kernel, skipping the first `skip` (warm-up) ones.
HBM-side bytes per dispatch: FETCH_SIZE and WRITE_SIZE are in KB.
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import sys


def summarise(root: str, kernel: str, skip: int = 3) -> dict:
    counters: dict[str, list[float]] = collections.defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        per_dispatch: dict[str, dict[str, float]] = collections.defaultdict(dict)
        order = []
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            d = r["Dispatch_Id"]
            if d not in per_dispatch:
                order.append(d)
            per_dispatch[d][r["Counter_Name"]] = float(r["Counter_Value"])
            meta = {"kernel": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                    "workgroup": int(r["Workgroup_Size"]), "vgpr": int(r["VGPR_Count"]),
                    "sgpr": int(r["SGPR_Count"]), "lds_bytes": int(r["LDS_Block_Size"])}
        for d in order[skip:]:
            for k, v in per_dispatch[d].items():
                counters[k].append(v)
    out = {"kernel": meta, "dispatches": {k: len(v) for k, v in counters.items()},
           "mean": {k: sum(v) / len(v) for k, v in counters.items() if v}}
    m = out["mean"]
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        out["hbm_bytes_per_dispatch"] = (m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
    if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_rate"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
        out["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    return out


if __name__ == "__main__":
    root, kern, path = sys.argv[1:4]
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    res = summarise(root, kern, skip)
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["mean"], indent=1))
