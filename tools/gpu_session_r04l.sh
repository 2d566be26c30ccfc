#!/bin/bash
# round 4 session l: pass B fail lists slot by slot (no select tree): parity,
# A/B against the ping-pong build
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/l_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/l_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="pp=tools/ab/libsketch_pp.so;tree=" ROUNDS=3 timeout -k 10 400 bash tools/ab_libs.sh > $O/r04_ab_pbslot.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pbslot.txt
