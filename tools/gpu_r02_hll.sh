#!/bin/bash
# line-owned PFADD (hll_mode 1) vs CAS (0): partitioned parity tests, then C3 bench + rocprof for each mode
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_k1_partitioned.py > gpurun_out/t_hll.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_hll.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/t_hll.log; exit $rc; fi
for m in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hll$m -o run --output-format csv -- python bench.py --config c3 --steps 20 --warmup 5 --no-cpu --streams 1 --graph 0 --hll-mode $m > gpurun_out/prof_hll$m.log 2>&1
  rc=$?; echo "mode $m rocprof rc=$rc"; tail -1 gpurun_out/prof_hll$m.log | cut -c1-400
  find gpurun_out/prof_hll$m -name "*kernel_stats.csv" -exec cat {} \; | grep part | cut -d, -f1-4
  if [ $rc -ne 0 ]; then exit $rc; fi
done
