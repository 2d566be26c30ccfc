#!/bin/bash
# round 5 session oo: the window pass's slice of a hot window (records per
# block before a window is cut): 32 k (default, klog 1), 16 k, 8 k
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 env SKE_LIB=tools/abv/libsketch_slice4096.so python -u -m pytest tests/test_seg_pfadd.py -x -q --timeout 300 --timeout-method thread > $O/r05oo_tests.log 2>&1; rc=$?
echo "tests (8 k slices) rc=$rc"; tail -2 $O/r05oo_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05oo_$tag.json 2> $O/r05oo_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05oo_$tag.err; exit 1; }; }
for i in 1 2; do
  run s32k_$i X=1
  run s16k_$i SKE_LIB=tools/abv/libsketch_slice8192.so
  run s8k_$i SKE_LIB=tools/abv/libsketch_slice4096.so
done
python tools/r05_passes.py $O/r05oo_*.json
