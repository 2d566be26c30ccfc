#!/bin/bash
# round 4 session ze: pass B with the units past the last whole round robin
# split evenly over the XCD's blocks (SKE_PB_TAIL) -- parity, then A/B
mkdir -p gpurun_out
SKE_LIB=tools/ab/libsketch_pbtail.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_k1_partitioned.py tests/test_full_size.py > gpurun_out/ze_pbtail_tests.log 2>&1
rc=$?; echo "pbtail tests rc=$rc"; tail -2 gpurun_out/ze_pbtail_tests.log; [ $rc -eq 0 ] || exit 1
LIBS="base=tools/ab/libsketch_base.so;pbtail=tools/ab/libsketch_pbtail.so" ROUNDS=4 bash tools/ab_libs.sh | tee gpurun_out/r04_ab_pb_tail.txt
