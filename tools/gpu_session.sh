#!/bin/bash
# One GPU session: parity tests, smoke, the default bench line (with the CPU
# baseline), a rocprofv3 kernel trace of the default bench, then the bench
# lines of $MATRIX (';'-separated argument sets) and, with STAMPS=1, the K1
# phase timeline.  Every GPU step has its own time limit; the first failure
# ends the session.
mkdir -p gpurun_out
export TMPDIR=/tmp
nproc > gpurun_out/host.txt; lscpu | grep -E "Model name|^CPU\(s\)" >> gpurun_out/host.txt
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu $PROF_ARGS > gpurun_out/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
IFS=';' read -ra SETS <<< "$MATRIX"
for v in "${SETS[@]}"; do
  timeout -k 10 300 python bench.py --no-cpu --secondary none $v > gpurun_out/bench_m.log 2>&1; rc=$?
  if [ $rc -ne 0 ]; then echo "bench [$v] rc=$rc"; tail -5 gpurun_out/bench_m.log; exit $rc; fi
  echo -n "[$v] "; python -c "import json; d=json.loads(open('gpurun_out/bench_m.log').read().strip().splitlines()[-1]); r=d['roofline']; print('%.3e swipes/s  step %.4f ms  kernel %s %.4f ms  enq %.1f us  %s frac=%.2f  passes %s' % (d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms'], d['host_enqueue_us_per_step'], d['config']['k1_variant'], r['frac'], {k: round(v['ms'], 4) for k, v in r['passes'].items()}))"
done
if [ -n "$STAMPS" ]; then
  for t in ${STAMP_TILES:-2}; do
    timeout -k 10 120 python tools/stamps/run_stamps.py $t > gpurun_out/stamps_$t.log 2>&1; rc=$?
    echo "stamps tile=$t rc=$rc"; cat gpurun_out/stamps_$t.log | tail -14
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
fi
exit 0
