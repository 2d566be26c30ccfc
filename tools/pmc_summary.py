"""Summarise rocprofv3 --pmc passes for one kernel into a JSON file.

usage: python tools/pmc_summary.py [--launch] [--wide F] <pmc_root_dir> <kernel-substring> <out.json> [skip]

Each sub-directory of <pmc_root_dir> is one rocprofv3 pass
(<pass>/run_counter_collection.csv).  Per counter the value is averaged over
the dispatches of the kernel, skipping the first `skip` (warm-up) ones.
HBM-side bytes per dispatch: FETCH_SIZE and WRITE_SIZE are in KB.

--wide F: the share F (0..1) of the kernel's fetched bytes that come from
16-B-per-lane streaming loads (pass B's probe records and LDS image: 1).  On
gfx950 FETCH_SIZE reports exactly half of such streams (MI355X_MICROARCH.md,
HBM section), so the corrected read bytes are FETCH_SIZE * (1 + F); the
summary keeps the raw value too ("hbm_bytes_per_dispatch" raw,
"hbm_bytes_corrected" with the correction).

--launch: the substring matches several kernels that together make one
launch of the path (the XCD-partitioned K1: hash, region and finish passes);
each counter is then the sum over those kernels of their per-dispatch means,
i.e. per launch, and the per-kernel means are kept under "per_kernel".
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import sys


def summarise(root: str, kernel: str, skip: int = 3, wide: float = 0.0) -> dict:
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
        out["fetch_wide_fraction"] = wide
        out["hbm_bytes_corrected"] = (m["FETCH_SIZE"] * (1.0 + wide) + m["WRITE_SIZE"]) * 1024
    if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_rate"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
        out["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    if "TCC_EA0_RDREQ_128B_sum" in m and "TCC_EA0_RDREQ_64B_sum" in m:
        # calibrated read bytes (tools/fetchcal.hip, profiles/r04_fetchcal.json): the
        # memory-side read requests by size, 128 / 64 / 32 B -- FETCH_SIZE counts every
        # request at 64 B, half of a 128-B line whatever the loads' width
        rd = (128 * m["TCC_EA0_RDREQ_128B_sum"] + 64 * m["TCC_EA0_RDREQ_64B_sum"]
              + 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0.0))
        out["read_bytes_by_request_size"] = rd
        if "WRITE_SIZE" in m:
            out["hbm_bytes_calibrated"] = rd + m["WRITE_SIZE"] * 1024
    return out


def summarise_launch(root: str, kernel: str, skip: int = 3) -> dict:
    names = set()
    for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                names.add(r["Kernel_Name"])
    per = {n: summarise(root, n, skip) for n in sorted(names)}
    mean: dict[str, float] = collections.defaultdict(float)
    for res in per.values():
        for k, v in res["mean"].items():
            mean[k] += v
    out = {"kernels": sorted(names), "mean": dict(mean),
           "per_kernel": {n: r["mean"] for n, r in per.items()}}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        out["hbm_bytes_per_dispatch"] = (mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
    if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
        out["l2_hit_rate"] = mean["TCC_HIT_sum"] / max(1.0, mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"])
    return out


if __name__ == "__main__":
    argv = sys.argv[1:]
    launch = "--launch" in argv
    if launch:
        argv.remove("--launch")
    wide = 0.0
    if "--wide" in argv:
        i = argv.index("--wide")
        wide = float(argv[i + 1])
        del argv[i:i + 2]
    root, kern, path = argv[:3]
    skip = int(argv[3]) if len(argv) > 3 else 3
    res = summarise_launch(root, kern, skip) if launch else summarise(root, kern, skip, wide)
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["mean"], indent=1))
