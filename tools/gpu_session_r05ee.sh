#!/bin/bash
# round 5 session ee: the new auto level-1 bucket rule -- segmented PFADD and
# partitioned parity tests, then the default bench twice and the shard once
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_seg_pfadd.py tests/test_full_size.py tests/test_k1_partitioned.py -x -q --timeout 300 --timeout-method thread > $O/r05ee_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/r05ee_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
for i in 1 2; do timeout -k 10 300 python -u bench.py $B > $O/r05ee_n1_$i.json 2> $O/r05ee_n1_$i.err || { echo "bench failed"; tail -5 $O/r05ee_n1_$i.err; exit 1; }; done
timeout -k 10 300 python -u bench.py $B --shard 8 > $O/r05ee_shard8.json 2> $O/r05ee_shard8.err || { echo "bench shard failed"; tail -5 $O/r05ee_shard8.err; exit 1; }
python tools/r05_passes.py $O/r05ee_*.json
