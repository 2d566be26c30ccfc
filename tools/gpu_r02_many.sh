#!/bin/bash
# partitioned-K1 parity after the pass A/B changes, then a kernel trace of the
# many-batch call (--persistent 1) against host launches (gaps between kernels)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_k1_partitioned.py tests/test_full_size.py > gpurun_out/many_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/many_tests.log; if [ $rc -ne 0 ]; then grep -B5 -A30 "^____" gpurun_out/many_tests.log | head -60; exit $rc; fi
for mode in host many; do
  extra=""; [ $mode = many ] && extra="--persistent 1"
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_$mode -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-check --pass-timing 0 $extra > gpurun_out/trace_$mode.log 2>&1
  rc=$?; echo "trace $mode rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/trace_$mode.log; exit $rc; fi
  grep '"value"' gpurun_out/trace_$mode.log | cut -c1-200
done
