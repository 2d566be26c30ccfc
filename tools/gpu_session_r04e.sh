#!/bin/bash
# round 4 session e: parity of the pass-A rewrite (DPP scan, v_bfe counter
# addresses), A/B against the dense build and r03, benches (default and
# --exchange 1) with kernel-trace stats, calibration (reads + writes), PMC
# passes of the partitioned K1 and of C2's LDS K1.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/e_tree.log 2>&1; rc=$?; echo "tree tests rc=$rc"; tail -3 $O/e_tree.log; [ $rc -eq 0 ] || exit $rc
LIBS="r03=tools/ab/libsketch_r03.so;dense=tools/ab/libsketch_dense.so;tree=" ROUNDS=2 timeout -k 10 400 bash tools/ab_libs.sh > $O/r04_ab_libs4.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_libs4.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py > $O/r04_bench2.json 2> $O/r04_bench2.err || { echo "bench failed"; tail -5 $O/r04_bench2.err; exit 1; }
echo "bench ok"; cut -c1-400 $O/r04_bench2.json
timeout -k 10 200 python -u bench.py --exchange 1 --secondary none --no-cpu > $O/r04_exch2.json 2> $O/r04_exch2.err || { echo "exch bench failed"; tail -5 $O/r04_exch2.err; exit 1; }
echo "exchange bench ok"; cut -c1-300 $O/r04_exch2.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ktx -o run --output-format csv -- python bench.py --exchange 1 --secondary none --no-cpu --no-check --pass-replay 0 > $O/ktx.log 2>&1 || { echo "ktx failed"; tail -5 $O/ktx.log; exit 1; }
echo "kernel trace (exchange) ok"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --secondary none --no-cpu --no-check --pass-replay 0 > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
echo "kernel trace ok"
timeout -k 10 300 bash tools/gpu_fetchcal.sh > $O/r04_fetchcal3.log 2>&1 || { echo "fetchcal failed"; tail -5 $O/r04_fetchcal3.log; exit 1; }
echo "fetchcal ok"
TAG=r04c3 timeout -k 10 600 bash tools/gpu_pmc_part.sh > $O/r04_pmc_part.log 2>&1 || { echo "pmc part failed"; tail -5 $O/r04_pmc_part.log; exit 1; }
echo "pmc part ok"
TAG=r04c2 timeout -k 10 600 bash tools/gpu_pmc_c2.sh > $O/r04_pmc_c2.log 2>&1 || { echo "pmc c2 failed"; tail -5 $O/r04_pmc_c2.log; exit 1; }
echo "pmc c2 ok"
