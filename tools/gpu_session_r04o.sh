#!/bin/bash
# round 4 session o: RCCL code paths at world 1 (collectives forced on) in the
# exchange and sharded-query tests, then the whole exchange / sharded files
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_exchange_gpu.py tests/test_sharded_gpu.py -v --timeout 120 --timeout-method thread > $O/o_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/o_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
