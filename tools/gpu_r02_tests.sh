#!/bin/bash
# the full -m gpu suite, one process, per-test timeouts
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|PASSED|FAILED|ERROR" gpurun_out/gpu_tests.log | tail -8
if [ $rc -ne 0 ]; then grep -B5 -A40 "^____" gpurun_out/gpu_tests.log | head -120; fi
exit $rc
