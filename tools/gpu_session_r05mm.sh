#!/bin/bash
# round 5 session mm: pass A's id prefetch two tiles ahead (ids load at the
# start of the tile before, from offsets loaded a tile earlier) vs one
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_k1_partitioned.py tests/test_seg_pfadd.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > $O/r05mm_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/r05mm_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05mm_$tag.json 2> $O/r05mm_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05mm_$tag.err; exit 1; }; }
for i in 1 2; do
  run new_$i X=1
  run base_$i SKE_LIB=tools/abv/libsketch_base.so
done
python tools/r05_passes.py $O/r05mm_*.json
