#!/bin/bash
# round 5 session c: segmented PFADD parity (cut windows), A/B at the shard and large batches
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_seg_pfadd.py -x -v --timeout 120 --timeout-method thread > $O/r05c_seg_tests.log 2>&1; rc=$?
echo "seg tests rc=$rc"; grep -E "PASS|FAIL|Error|error" $O/r05c_seg_tests.log | tail -22 | cut -c1-200; [ $rc -eq 0 ] || exit $rc
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --secondary none "$@" > $O/r05c_$n.json 2> $O/r05c_$n.err || { echo "$n failed"; tail -5 $O/r05c_$n.err; exit 1; }
  python tools/r05_passes.py $O/r05c_$n.json
}
run shard8_seg --shard 8 --opt hll_seg=1
run shard8_seg_k2 --shard 8 --opt hll_seg=1 --opt seg_klog=2
run b128m_seg --batch 134217728 --steps 4 --warmup 2 --opt hll_seg=1
run b128m_seg_k2 --batch 134217728 --steps 4 --warmup 2 --opt hll_seg=1 --opt seg_klog=2
