#!/bin/bash
# round 4 session y: pass C three-stage pipeline (pre-check loads a tile
# ahead, CASes settled a tile later): parity + A/B
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
SKE_LIB=tools/ab/libsketch_pcpipe.so timeout -k 10 400 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/y_tests.log 2>&1; rc=$?; echo "pcpipe tests rc=$rc"; tail -1 $O/y_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="tree=;pcpipe=tools/ab/libsketch_pcpipe.so" ROUNDS=3 timeout -k 10 400 bash tools/ab_libs.sh > $O/r04_ab_pcpipe.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pcpipe.txt
