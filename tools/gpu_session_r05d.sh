#!/bin/bash
# round 5 session d: segmented PFADD parity (cut windows), A/B at the shard and large batches
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_seg_pfadd.py -x -v --timeout 120 --timeout-method thread > $O/r05d_seg_tests.log 2>&1; rc=$?
echo "seg tests rc=$rc"; grep -E "PASS|FAIL|Error|error" $O/r05d_seg_tests.log | tail -22 | cut -c1-200; [ $rc -eq 0 ] || exit $rc
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --secondary none "$@" > $O/r05d_$n.json 2> $O/r05d_$n.err || { echo "$n failed"; tail -5 $O/r05d_$n.err; exit 1; }
  python tools/r05_passes.py $O/r05d_$n.json
}
run shard8_seg --shard 8 --opt hll_seg=1
run shard8_seg_k2 --shard 8 --opt hll_seg=1 --opt seg_klog=2
run b128m_seg --batch 134217728 --steps 4 --warmup 2 --opt hll_seg=1
run b128m_seg_k2 --batch 134217728 --steps 4 --warmup 2 --opt hll_seg=1 --opt seg_klog=2
timeout -k 10 400 python -u bench.py --no-cpu --secondary none --config c5 --steps 5 --warmup 2 > $O/r05d_c5.json 2> $O/r05d_c5.err || { echo "c5 failed"; tail -5 $O/r05d_c5.err; exit 1; }
python -c "import json; d=json.loads(open('$O/r05d_c5.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d.get('rollup'))[:900]); print(json.dumps(d.get('host_fed'))[:600])"
