#!/bin/bash
# GPU session: parity tests, then one bench line per argument set in $MATRIX
# (';'-separated), then a rocprofv3 kernel-trace of the default bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
IFS=';' read -ra SETS <<< "$MATRIX"
for v in "${SETS[@]}"; do
  timeout -k 10 300 python bench.py --no-cpu $v > gpurun_out/bench_m.log 2>&1; rc=$?
  if [ $rc -ne 0 ]; then echo "bench [$v] rc=$rc"; tail -5 gpurun_out/bench_m.log; exit $rc; fi
  echo -n "[$v] "; python -c "import json; d=json.loads(open('gpurun_out/bench_m.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%.3e swipes/s  step %.4f ms  kernel %.4f ms  %s tile=%s frac=%.2f' % (d['value'], d['ms_per_step'], r['kernel_ms'], d['config']['k1_variant'], d['config']['tile'], r['frac']))"
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; grep -m1 "k_swipes<0" gpurun_out/prof/run_kernel_stats.csv | cut -d, -f2-5 
fi
exit 0
