#!/bin/bash
# round 4 session w: pass C 1024 x 1 as the default (parity), and 2 blocks per
# CU (each 4 runs) against 8 (all 2048 blocks one run each): A/B with the
# previous default build (256 x 4)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > $O/w_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/w_tests.log; [ $rc -eq 0 ] || exit $rc
SKE_LIB=tools/ab/libsketch_pcg2.so timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py -q --timeout 120 --timeout-method thread > $O/w_pcg2.log 2>&1; rc=$?; echo "pcg2 tests rc=$rc"; tail -1 $O/w_pcg2.log; [ $rc -eq 0 ] || exit $rc
LIBS="pp=tools/ab/libsketch_pp.so;tree=;pcg2=tools/ab/libsketch_pcg2.so" ROUNDS=3 timeout -k 10 500 bash tools/ab_libs.sh > $O/r04_ab_pcgrid.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pcgrid.txt
