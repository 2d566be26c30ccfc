#!/bin/bash
# round 4 session g: full parity suite, smoke, exchange bench + kernel trace,
# default bench + kernel trace
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r04_gpu_tests3.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -5 $O/r04_gpu_tests3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r04_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 $O/r04_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --exchange 1 --secondary none --no-cpu > $O/r04_exch4.json 2> $O/r04_exch4.err || { echo "exch bench failed"; tail -5 $O/r04_exch4.err; exit 1; }
echo "exchange bench ok"; cut -c1-300 $O/r04_exch4.json
rm -rf $O/ktx $O/kt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ktx -o run --output-format csv -- python bench.py --exchange 1 --secondary none --no-cpu --no-check --pass-replay 0 > $O/ktx.log 2>&1 || { echo "ktx failed"; tail -5 $O/ktx.log; exit 1; }
timeout -k 10 200 python -u bench.py > $O/r04_bench4.json 2> $O/r04_bench4.err || { echo "bench failed"; tail -5 $O/r04_bench4.err; exit 1; }
echo "bench ok"; cut -c1-300 $O/r04_bench4.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --secondary none --no-cpu --no-check --pass-replay 0 > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
echo "traces ok"
