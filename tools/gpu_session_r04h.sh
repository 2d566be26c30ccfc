#!/bin/bash
# round 4 session h: packed route words (exchange tests, --exchange 1 bench +
# kernel trace), pass B sweep A/B on this box, pass tests of the cleaned build
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_exchange_gpu.py tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/h_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/h_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --exchange 1 --secondary none --no-cpu > $O/r04_exch5.json 2> $O/r04_exch5.err || { echo "exch bench failed"; tail -5 $O/r04_exch5.err; exit 1; }
echo "exchange bench ok"; cut -c1-300 $O/r04_exch5.json
rm -rf $O/ktx
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ktx -o run --output-format csv -- python bench.py --exchange 1 --secondary none --no-cpu --no-check --pass-replay 0 > $O/ktx.log 2>&1 || { echo "ktx failed"; tail -5 $O/ktx.log; exit 1; }
echo "kernel trace ok"
LIBS="tree=;sp1=tools/ab/libsketch_sp1.so" ROUNDS=3 timeout -k 10 400 bash tools/ab_libs.sh > $O/r04_ab_sp.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_sp.txt
