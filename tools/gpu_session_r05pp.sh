#!/bin/bash
# round 5 session pp: the window pass's slice, larger: 32 k (default, klog 1), 64 k, 128 k
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 env SKE_LIB=tools/abv/libsketch_slice65536.so python -u -m pytest tests/test_seg_pfadd.py -x -q --timeout 300 --timeout-method thread > $O/r05pp_tests.log 2>&1; rc=$?
echo "tests (128 k slices) rc=$rc"; tail -2 $O/r05pp_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05pp_$tag.json 2> $O/r05pp_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05pp_$tag.err; exit 1; }; }
for i in 1 2; do
  run s32k_$i X=1
  run s64k_$i SKE_LIB=tools/abv/libsketch_slice32768.so
  run s128k_$i SKE_LIB=tools/abv/libsketch_slice65536.so
done
python tools/r05_passes.py $O/r05pp_*.json
