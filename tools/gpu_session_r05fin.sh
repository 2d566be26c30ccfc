#!/bin/bash
# round 5 final session: the final tree -- full GPU suite, smoke, PMC passes, default bench line, kernel trace
# default bench line and its kernel trace
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05fin_gpu_tests.log 2>&1; rc=$?
echo "gpu suite rc=$rc"; tail -2 $O/r05fin_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r05fin_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/r05fin_smoke.log; [ $rc -eq 0 ] || exit $rc
rm -rf $O/pmc_r05 $O/pmc_r05_*.json
NSUB=4 STEP_SWIPES=134217728 bash tools/gpu_pmc_r05.sh > $O/r05fin_pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/r05fin_pmc.log; exit 1; }
tail -5 $O/r05fin_pmc.log
timeout -k 10 400 python -u bench.py > $O/r05fin_bench.json 2> $O/r05fin_bench.err || { echo "bench failed"; tail -5 $O/r05fin_bench.err; exit 1; }
python tools/r05_passes.py $O/r05fin_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r05fin_trace -o run --output-format csv -- python bench.py --no-cpu --secondary none --host-fed 0 > $O/r05fin_trace.log 2>&1 || { echo "trace failed"; tail -5 $O/r05fin_trace.log; exit 1; }
echo trace ok
