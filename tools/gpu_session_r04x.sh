#!/bin/bash
# round 4 session x: final confirmation -- full parity suite, smoke, default
# bench, kernel trace, pass PMC, the config matrix
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r04_gpu_tests6.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -2 $O/r04_gpu_tests6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r04_smoke3.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/r04_smoke3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py > $O/r04_bench8.json 2> $O/r04_bench8.err || { echo "bench failed"; tail -5 $O/r04_bench8.err; exit 1; }
echo "bench ok"; cut -c1-220 $O/r04_bench8.json
rm -rf $O/kt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --secondary none --no-cpu --no-check --pass-replay 0 > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
echo "trace ok"
rm -rf $O/pmc_r04c3h
TAG=r04c3h timeout -k 10 600 bash tools/gpu_pmc_part.sh > $O/r04_pmc_part4.log 2>&1 || { echo "pmc failed"; tail -5 $O/r04_pmc_part4.log; exit 1; }
echo "pmc ok"
SKIP_TESTS=1 SKIP_BENCH=1 MATRIX="--config c1;--config c2;--config c4;--config c5;--config c3 --steps 200;--exchange 1" timeout -k 10 900 bash tools/gpu_session.sh > $O/r04_matrix2.txt 2>&1; rc=$?; echo "matrix rc=$rc"; grep "^\[" $O/r04_matrix2.txt
