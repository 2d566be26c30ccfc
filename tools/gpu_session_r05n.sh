#!/bin/bash
# round 5 session n: full parity suite, smoke, the default bench line, kernel trace
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05n_gpu_tests.log 2>&1; rc=$?
echo "gpu suite rc=$rc"; tail -3 $O/r05n_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r05n_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/r05n_bench.json 2> $O/r05n_bench.err || { echo "bench failed"; tail -5 $O/r05n_bench.err; exit 1; }
python tools/r05_passes.py $O/r05n_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r05n_trace -o run --output-format csv -- python bench.py --no-cpu --secondary none --host-fed 0 > $O/r05n_trace.log 2>&1 || { echo "trace failed"; tail -5 $O/r05n_trace.log; exit 1; }
echo trace ok
