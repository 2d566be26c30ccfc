#!/bin/bash
# round 4 session j: pass-B VALU trims (raw v_bfe bit tests, one-sided lower
# bound of the in-run mask): parity + A/B against the previous build
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/j_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/j_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="prev=tools/ab/libsketch_prev.so;tree=" ROUNDS=3 timeout -k 10 400 bash tools/ab_libs.sh > $O/r04_ab_pbvalu.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pbvalu.txt
