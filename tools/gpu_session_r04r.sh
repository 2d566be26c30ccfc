#!/bin/bash
# round 4 session r: pass B loads the next unit's image during the last round
# (prefetch into registers): parity + A/B against the previous build
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > $O/r_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/r_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="pp=tools/ab/libsketch_pp.so;tree=" ROUNDS=3 timeout -k 10 400 bash tools/ab_libs.sh > $O/r04_ab_pbpref.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pbpref.txt
