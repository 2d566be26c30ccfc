#!/bin/bash
# round 5 session bb: the full GPU suite and smoke on the late-round-5 tree
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05bb_gpu_tests.log 2>&1; rc=$?
echo "gpu suite rc=$rc"; tail -3 $O/r05bb_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r05bb_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/r05bb_smoke.log; exit $rc
