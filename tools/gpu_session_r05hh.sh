#!/bin/bash
# round 5 session hh: sub-batches of up to 2^26 swipes (pass B's record range
# per XCD tile group, D's run staging capped), window passes per group of
# sub-batches; parity tests, then A/B 2^26 (default) vs 2^25, two alternations
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_seg_pfadd.py tests/test_k1_partitioned.py tests/test_full_size.py tests/test_rec_groups.py -x -q --timeout 300 --timeout-method thread > $O/r05hh_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/r05hh_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B > $O/r05hh_s64_$i.json 2> $O/r05hh_s64_$i.err || { echo "bench s64 failed"; tail -5 $O/r05hh_s64_$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py $B --part-sub 33554432 > $O/r05hh_s32_$i.json 2> $O/r05hh_s32_$i.err || { echo "bench s32 failed"; tail -5 $O/r05hh_s32_$i.err; exit 1; }
done
python tools/r05_passes.py $O/r05hh_s*.json
