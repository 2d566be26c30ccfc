#!/bin/bash
# round 5 session vv: window pass at klog 1 with 3 blocks per CU (80 VGPRs, no
# spill) and 4 or 8 records per thread per round, vs 4 blocks (64 VGPRs)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 env SKE_LIB=tools/abv/libsketch_e34.so python -u -m pytest tests/test_seg_pfadd.py -x -q --timeout 300 --timeout-method thread > $O/r05vv_tests.log 2>&1; rc=$?
echo "tests (3 blocks) rc=$rc"; tail -2 $O/r05vv_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05vv_$tag.json 2> $O/r05vv_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05vv_$tag.err; exit 1; }; }
for i in 1 2; do
  run b4r4_$i X=1
  run b3r4_$i SKE_LIB=tools/abv/libsketch_e34.so
  run b3r8_$i SKE_LIB=tools/abv/libsketch_e38.so
done
python tools/r05_passes.py $O/r05vv_*.json
