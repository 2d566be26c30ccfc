#!/bin/bash
# round 4 session u: pass C block shapes (512 x 2 swipes, 128 x 8, 4 blocks per
# CU): parity of the changed shapes + A/B
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
for v in pc512 pc128; do
  SKE_LIB=tools/ab/libsketch_$v.so timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py -q --timeout 120 --timeout-method thread > $O/u_$v.log 2>&1; rc=$?; echo "$v tests rc=$rc"; tail -1 $O/u_$v.log; [ $rc -eq 0 ] || exit $rc
done
LIBS="tree=;pc512=tools/ab/libsketch_pc512.so;pc128=tools/ab/libsketch_pc128.so;pcg4=tools/ab/libsketch_pcg4.so" ROUNDS=2 timeout -k 10 500 bash tools/ab_libs.sh > $O/r04_ab_pcshape.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pcshape.txt
