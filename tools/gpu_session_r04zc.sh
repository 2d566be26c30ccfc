#!/bin/bash
# round 4 session zc: closing check of the committed tree -- full parity
# suite, smoke, default bench line
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r04_gpu_tests7.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -2 $O/r04_gpu_tests7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r04_smoke4.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/r04_smoke4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py > $O/r04_bench9.json 2> $O/r04_bench9.err || { echo "bench failed"; tail -5 $O/r04_bench9.err; exit 1; }
echo "bench ok"; cut -c1-300 $O/r04_bench9.json
