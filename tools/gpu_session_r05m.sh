#!/bin/bash
# round 5 session m: window pass with LDS-DMA images + coalesced records -- parity, A/B
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_seg_pfadd.py -x -q --timeout 120 --timeout-method thread > $O/r05m_seg_tests.log 2>&1; rc=$?
echo "seg tests rc=$rc"; tail -3 $O/r05m_seg_tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --secondary none --host-fed 0 "$@" > $O/r05m_$n.json 2> $O/r05m_$n.err || { echo "$n failed"; tail -5 $O/r05m_$n.err; exit 1; }
  python tools/r05_passes.py $O/r05m_$n.json
}
for k in 0 1 2 3; do
  run b128m_k$k --batch 134217728 --steps 4 --warmup 2 --opt hll_seg=1 --opt seg_klog=$k
done
for k in 1 2; do
  run shard8_b128m_k$k --shard 8 --batch 134217728 --steps 4 --warmup 2 --opt hll_seg=1 --opt seg_klog=$k
done
run shard8_k1 --shard 8 --opt hll_seg=1 --opt seg_klog=1
