#!/bin/bash
# round 4: dense pair runs (kAlign 1) as the product pass A, A/B against r03
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/d_tree.log 2>&1; rc=$?; echo "tree tests rc=$rc"; tail -3 $O/d_tree.log; [ $rc -eq 0 ] || exit $rc
SKE_LIB=tools/ab/libsketch_wpe6.so timeout -k 10 200 python -u -m pytest tests/test_k1_partitioned.py -q --timeout 120 --timeout-method thread > $O/d_wpe6.log 2>&1; echo "wpe6 tests rc=$?"; tail -3 $O/d_wpe6.log
LIBS="r03=tools/ab/libsketch_r03.so;a4nu=tools/ab/libsketch_a4nu.so;tree=;dunroll=tools/ab/libsketch_dunroll.so;a4s=tools/ab/libsketch_a4s.so;dnosplit=tools/ab/libsketch_dnosplit.so;wpe6=tools/ab/libsketch_wpe6.so" ROUNDS=2 timeout -k 10 700 bash tools/ab_libs.sh > $O/r04_ab_libs3.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_libs3.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r04_gpu_tests2.log 2>&1; echo "gpu suite rc=$?"; tail -5 $O/r04_gpu_tests2.log
