#!/bin/bash
# non-temporal policies: partitioned-K1 parity with the nt passes, the default
# bench, then the C5 rollups with and without nt register loads (A/B)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_k1_partitioned.py tests/test_full_size.py > gpurun_out/nt_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/nt_tests.log; if [ $rc -ne 0 ]; then grep -B5 -A30 "^____" gpurun_out/nt_tests.log | head -60; exit $rc; fi
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/nt_bench.json 2> gpurun_out/nt_bench.err || { tail -5 gpurun_out/nt_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/nt_bench.json').read().strip().splitlines()[-1]); p=d['roofline']['passes']
print('bench %.4e ms/step %.4f' % (d['value'], d['ms_per_step']), {k: round(v['ms'], 4) for k, v in p.items()}, d['check']['ok'])"
for r in 1 2; do
  for lib in real-time-student-attendance-system_amd/csrc/libsketch.so tools/ab/libsketch_k2nt.so; do
    SKE_LIB=$lib timeout -k 10 300 python tools/bench_rollup.py --swipes 160000000 > gpurun_out/nt_roll.json 2> gpurun_out/nt_roll.err || { tail -5 gpurun_out/nt_roll.err; exit 1; }
    echo "$(basename $lib) $(tail -1 gpurun_out/nt_roll.json | cut -c1-600)"
  done
done
# the LDS K1 (C2) with nt swipe streams
for r in 1 2; do
  for lib in real-time-student-attendance-system_amd/csrc/libsketch.so tools/ab/libsketch_k1nt3.so tools/ab/libsketch_k1nt7.so; do
    SKE_LIB=$lib timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu --no-check > gpurun_out/nt_c2.json 2> gpurun_out/nt_c2.err || { tail -5 gpurun_out/nt_c2.err; exit 1; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/nt_c2.json').read().strip().splitlines()[-1])
print(sys.argv[1], 'c2 %.4e/s ms/step %.5f kernel %.5f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms']))" $(basename $lib)
  done
done
