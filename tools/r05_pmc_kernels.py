"""Per-kernel PMC means (per dispatch, warm-up dispatches skipped) from
tools/gpu_pmc_ab.sh passes, calibrated HBM bytes = read requests x their
size + WRITE_SIZE (tools/fetchcal.hip), for the kernels named.
usage: python tools/r05_pmc_kernels.py <out.json> <kernel-substr,...> <tag>=<dir> ...
"""
import collections
import csv
import glob
import json
import os
import sys

SKIP = 2 * 8  # the bench's 2 warm-up steps x 8 sub-batches


def kernel_means(root, subs):
    acc = {s: collections.defaultdict(list) for s in subs}
    for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        rows, names = collections.defaultdict(dict), {}
        for r in csv.DictReader(open(f)):
            rows[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for s in subs:
            ds = [rows[d] for d in sorted(rows, key=int) if s in names[d]][SKIP:]
            for d in ds:
                for c, v in d.items():
                    acc[s][c].append(v)
    out = {}
    for s, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items() if v}
        o = {"mean": m, "dispatches": {c: len(v) for c, v in cs.items()}}
        if "TCC_EA0_RDREQ_128B_sum" in m:
            rd = 128 * m["TCC_EA0_RDREQ_128B_sum"] + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + \
                32 * m.get("TCC_EA0_RDREQ_32B_sum", 0)
            o["read_bytes_by_request_size"] = rd
            if "WRITE_SIZE" in m:
                o["write_bytes"] = m["WRITE_SIZE"] * 1024
                o["hbm_bytes_calibrated"] = rd + m["WRITE_SIZE"] * 1024
        out[s] = o
    return out


res = {}
subs = sys.argv[2].split(",")
for a in sys.argv[3:]:
    tag, d = a.split("=", 1)
    res[tag] = kernel_means(d, subs)
    for s in subs:
        o = res[tag][s]
        print("%-10s %-12s read %.3f GB  write %.3f GB  calibrated %.3f GB" % (
            tag, s, o.get("read_bytes_by_request_size", 0) / 1e9, o.get("write_bytes", 0) / 1e9,
            o.get("hbm_bytes_calibrated", 0) / 1e9))
json.dump(res, open(sys.argv[1], "w"), indent=1)
