#!/bin/bash
# GPU session: parity tests, bench (default + variants), rocprofv3 kernel stats.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for v in "" "--variant 0" "--probe-batch 4" "--variant 0 --probe-batch 4"; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu $v > gpurun_out/bench_v.log 2>&1; rc=$?
  echo "bench [$v] rc=$rc"; tail -1 gpurun_out/bench_v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['k1_variant'])"
  if [ $rc -ne 0 ]; then cat gpurun_out/bench_v.log | tail -5; exit $rc; fi
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
