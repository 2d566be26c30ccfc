#!/bin/bash
# round 5 session b: segmented PFADD parity, then A/B at the shard and large batches
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
true; rc=0

run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --secondary none "$@" > $O/r05b_$n.json 2> $O/r05b_$n.err || { echo "$n failed"; tail -5 $O/r05b_$n.err; exit 1; }
  python tools/r05_passes.py $O/r05b_$n.json
}
run shard8_off --shard 8 --opt hll_seg=0
run shard8_seg --shard 8 --opt hll_seg=1
run shard8_seg_k2 --shard 8 --opt hll_seg=1 --opt seg_klog=2
run b64m_seg --batch 67108864 --steps 6 --warmup 2 --opt hll_seg=1
run b128m_seg --batch 134217728 --steps 4 --warmup 2 --opt hll_seg=1
run b128m_seg_k2 --batch 134217728 --steps 4 --warmup 2 --opt hll_seg=1 --opt seg_klog=2
