"""PFADD-form A/B table from tools/gpu_pmc_ab.sh passes: per timed step (the
bench's 4 steps after 2 warm-up steps), the HBM read bytes by request size,
WRITE_SIZE and memory-side atomics of the PFADD side (CAS: k_part_c_fl;
segmented: k_seg_c1 + k_seg_scan + k_seg_d + the window pass k_seg_e E1/E2 +
k_seg_m) and of the whole K1 step.
usage: python tools/r05_pmc_ab.py <out.json> <tag>=<dir> ...
"""
import collections
import csv
import glob
import json
import os
import sys

PFADD = ("k_part_c_fl", "k_seg_")
WARM, STEPS = 2, 4


def per_step(root):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        rows = collections.defaultdict(dict)
        names = {}
        for r in csv.DictReader(open(f)):
            rows[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        by_kernel = collections.defaultdict(list)
        for d in sorted(rows, key=int):
            by_kernel[names[d]].append(rows[d])
        for k, ds in by_kernel.items():
            if not any(s in k for s in ("k_part_", "k_seg_")):
                continue
            ds = ds[len(ds) * WARM // (WARM + STEPS):]
            for d in ds:
                for c, v in d.items():
                    tot[k][c] += v / STEPS
    return tot


def row(tot, sel):
    m = collections.defaultdict(float)
    for k, cs in tot.items():
        if sel(k):
            for c, v in cs.items():
                m[c] += v
    rd = 128 * m["TCC_EA0_RDREQ_128B_sum"] + 64 * m["TCC_EA0_RDREQ_64B_sum"] + 32 * m["TCC_EA0_RDREQ_32B_sum"]
    return {"read_GB": rd / 1e9, "write_GB": m["WRITE_SIZE"] * 1024 / 1e9, "rdreq_128B_M": m["TCC_EA0_RDREQ_128B_sum"] / 1e6,
            "atomics_M": m["TCC_EA0_ATOMIC_sum"] / 1e6, "l2_miss_M": m["TCC_MISS_sum"] / 1e6}


out = {}
for a in sys.argv[2:]:
    tag, root = a.split("=", 1)
    tot = per_step(root)
    out[tag] = {"pfadd": row(tot, lambda k: any(s in k for s in PFADD)), "step": row(tot, lambda k: True)}
    p, s = out[tag]["pfadd"], out[tag]["step"]
    print("%-16s pfadd: rd %.3f GB wr %.3f GB atom %.2f M | step: rd %.3f wr %.3f GB" % (
        tag, p["read_GB"], p["write_GB"], p["atomics_M"], s["read_GB"], s["write_GB"]))
json.dump({"what": "per timed step (4 steps after 2 warm-up), rocprofv3 --pmc, tools/gpu_pmc_ab.sh", "forms": out},
          open(sys.argv[1], "w"), indent=1)
