#!/bin/bash
# round 5 session xx: D claiming its chunks from a counter
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_seg_pfadd.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > $O/r05xx_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/r05xx_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05xx_$tag.json 2> $O/r05xx_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05xx_$tag.err; exit 1; }; }
for i in 1 2; do
  run new_$i X=1
  run base_$i SKE_LIB=tools/abv/libsketch_base.so
done
B="$B --shard 8"
run shnew X=1
run shbase SKE_LIB=tools/abv/libsketch_base.so
python tools/r05_passes.py $O/r05xx_*.json
