#!/bin/bash
# round 4 session s: pass A waits for its counting atomics once per tile (after
# the last swipe) instead of once per swipe: parity + A/B
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
SKE_LIB=tools/ab/libsketch_wl.so timeout -k 10 400 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/s_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/s_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="tree=;wl=tools/ab/libsketch_wl.so" ROUNDS=3 timeout -k 10 400 bash tools/ab_libs.sh > $O/r04_ab_pawait.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pawait.txt
