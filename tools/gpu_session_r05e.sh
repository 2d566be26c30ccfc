#!/bin/bash
# round 5 session e: kernel trace of the segmented PFADD (E1 / E2 / M split)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
tr() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r05e_$n -o run --output-format csv -- python bench.py --no-cpu --no-check --secondary none --host-fed 0 "$@" > $O/r05e_$n.log 2>&1 || { echo "$n failed"; tail -5 $O/r05e_$n.log; exit 1; }
  f=$(find $O/r05e_$n -name "*kernel_stats.csv" | head -1)
  echo "== $n"; python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print("%-60s calls=%5s avg_us=%9.2f tot_ms=%8.3f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
}
tr shard8_k2 --shard 8 --opt hll_seg=1 --opt seg_klog=2 --steps 10 --warmup 2
tr b128m_k2 --batch 134217728 --opt hll_seg=1 --opt seg_klog=2 --steps 3 --warmup 1
