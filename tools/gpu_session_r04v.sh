#!/bin/bash
# round 4 session v: pass C at 512 x 2 and 1024 x 1 swipes per thread: A/B
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
SKE_LIB=tools/ab/libsketch_pc1024.so timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py -q --timeout 120 --timeout-method thread > $O/v_pc1024.log 2>&1; rc=$?; echo "pc1024 tests rc=$rc"; tail -1 $O/v_pc1024.log; [ $rc -eq 0 ] || exit $rc
LIBS="tree=;pc512=tools/ab/libsketch_pc512.so;pc1024=tools/ab/libsketch_pc1024.so" ROUNDS=3 timeout -k 10 500 bash tools/ab_libs.sh > $O/r04_ab_pcshape2.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pcshape2.txt
