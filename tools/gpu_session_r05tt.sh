#!/bin/bash
# round 5 session tt: pass B's work split 3 (units round robin while whole,
# the rest in equal (unit, 8-tile group) shares) vs 2 (round robin to the end)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 env SKE_LIB=tools/abv/libsketch_split3.so python -u -m pytest tests/test_k1_partitioned.py tests/test_seg_pfadd.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > $O/r05tt_tests.log 2>&1; rc=$?
echo "tests (split 3) rc=$rc"; tail -2 $O/r05tt_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05tt_$tag.json 2> $O/r05tt_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05tt_$tag.err; exit 1; }; }
for i in 1 2 3; do
  run s2_$i X=1
  run s3_$i SKE_LIB=tools/abv/libsketch_split3.so
done
B="$B --shard 8"; run sh2 X=1
run sh3 SKE_LIB=tools/abv/libsketch_split3.so
python tools/r05_passes.py $O/r05tt_*.json
