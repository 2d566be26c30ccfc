#!/bin/bash
# round 4 session k: pass B round ping-pong + v_bfm masks: parity, A/B against
# the previous two builds, then the config matrix on the final build
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/k_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/k_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="prev=tools/ab/libsketch_prev.so;b1=tools/ab/libsketch_b1.so;tree=" ROUNDS=3 timeout -k 10 500 bash tools/ab_libs.sh > $O/r04_ab_pbvalu2.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pbvalu2.txt
