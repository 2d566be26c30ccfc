#!/bin/bash
# round 5 session l: batch sweep of the segmented form (2-key windows) vs CAS
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --secondary none --host-fed 0 "$@" > $O/r05l_$n.json 2> $O/r05l_$n.err || { echo "$n failed"; tail -5 $O/r05l_$n.err; exit 1; }
  python tools/r05_passes.py $O/r05l_$n.json
}
run b64m_seg --batch 67108864 --steps 8 --warmup 2 --opt hll_seg=1 --opt seg_klog=1
run b256m_seg --batch 268435456 --steps 4 --warmup 2 --opt hll_seg=1 --opt seg_klog=1
run b256m_cas --batch 268435456 --steps 4 --warmup 2 --opt hll_seg=0
run b128m_seg20 --batch 134217728 --steps 20 --warmup 5 --opt hll_seg=1 --opt seg_klog=1
run shard8_b128m_seg --shard 8 --batch 134217728 --steps 8 --warmup 2 --opt hll_seg=1 --opt seg_klog=1
run shard8_b128m_cas --shard 8 --batch 134217728 --steps 8 --warmup 2 --opt hll_seg=0
