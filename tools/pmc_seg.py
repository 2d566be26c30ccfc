"""Per-kernel PMC summaries of the default C3 step (partitioned K1 +
segmented PFADD) from tools/gpu_pmc_seg.sh's passes, named by bench.py's pass
kinds: k_part_a, k_part_b, k_part_c (the segmented C1, k_seg_c1), k_seg_d
(k_seg_da per sub-batch; SEG_ARENA=0: k_seg_scan + k_seg_d), k_seg_e (window pass E1 + E2 + merge
M, per step).  Warm-up dispatches are skipped (2 steps of NSUB sub-batches;
env NSUB, default 4: 2^27 swipes in sub-batches of 2^25).  Every summary
records the swipes one launch covers (env STEP_SWIPES / NSUB; the window pass:
a step), so bench.py applies it only to launches of that size.
usage: NSUB=4 STEP_SWIPES=134217728 python tools/pmc_seg.py <pmc_root> <out_prefix>
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402

root, prefix = sys.argv[1], sys.argv[2]
NSUB = int(os.environ.get("NSUB", "4"))
STEP = int(os.environ.get("STEP_SWIPES", str(1 << 27)))
SKIP_SUB, SKIP_STEP = 2 * NSUB, 2
ROUND6 = os.environ.get("SEG_D_TEMPLATE", "1") == "1"  # round 6: k_seg_d<T> (round 5: k_seg_d(SegArgs))
plan = {"k_part_a": (["k_part_a3"], SKIP_SUB), "k_part_b": (["k_part_b"], SKIP_SUB),
        "k_part_c": (["k_seg_c1"], SKIP_SUB), "k_seg_d": (["k_seg_scan", "k_seg_d<" if ROUND6 else "k_seg_d("], SKIP_SUB),
        "k_seg_e": (["k_seg_e<1, false>", "k_seg_e<1, true>", "k_seg_m<1>"], SKIP_STEP)}
if os.environ.get("SEG_ARENA", "1") == "1":  # the arena form (default): D alone (k_seg_da), no scan pass
    plan["k_seg_d"] = (["k_seg_da<"], SKIP_SUB)
for name, (kernels, skip) in plan.items():
    parts = {k: summarise(root, k, skip) for k in kernels}
    mean = {}
    for p in parts.values():
        for c, v in p["mean"].items():
            mean[c] = mean.get(c, 0.0) + v
    out = {"kernels": {k: p["kernel"] for k, p in parts.items()}, "per_kernel": parts, "mean": mean,
           "what": "per launch of the pass (sum of its kernels' per-dispatch means)",
           "swipes_per_launch": STEP if skip == SKIP_STEP else STEP // NSUB}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        out["hbm_bytes_per_dispatch"] = (mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
    if "TCC_EA0_RDREQ_128B_sum" in mean and "WRITE_SIZE" in mean:
        rd = (128 * mean["TCC_EA0_RDREQ_128B_sum"] + 64 * mean["TCC_EA0_RDREQ_64B_sum"]
              + 32 * mean.get("TCC_EA0_RDREQ_32B_sum", 0.0))
        out["read_bytes_by_request_size"] = rd
        out["hbm_bytes_calibrated"] = rd + mean["WRITE_SIZE"] * 1024
    if mean.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_rate"] = mean.get("SQ_LDS_BANK_CONFLICT", 0.0) / mean["SQ_LDS_IDX_ACTIVE"]
    json.dump(out, open(prefix + name + ".json", "w"), indent=1)
    print(name, "calibrated GB %.3f" % (out.get("hbm_bytes_calibrated", 0) / 1e9),
          {k: round(v / 1e6, 2) for k, v in mean.items() if k.startswith("TCC_EA0") or k.startswith("SQ_INSTS_VALU")})
