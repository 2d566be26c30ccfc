#!/bin/bash
# round 5 session q: the group layout of pass A's records (option rec_groups):
# parity tests, then A/B of the default bench line, three alternations
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rec_groups.py tests/test_k1_partitioned.py tests/test_seg_pfadd.py -x -q --timeout 200 --timeout-method thread > $O/r05q_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/r05q_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 300 python -u bench.py --no-cpu --secondary none --host-fed 0 --opt rec_groups=$g > $O/r05q_g${g}_$i.json 2> $O/r05q_g${g}_$i.err || { echo "bench g$g failed"; tail -5 $O/r05q_g${g}_$i.err; exit 1; }
  done
done
python tools/r05_passes.py $O/r05q_g*_*.json
