#!/bin/bash
# persistent LDS K1 (C2): parity tests, then the C2 bench (persistent vs forked graph) under rocprof
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_full_size.py -k "c2" > gpurun_out/t_c2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_c2.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/t_c2.log; exit $rc; fi
timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu > gpurun_out/c2_pers.json 2> gpurun_out/c2_pers.err
rc=$?; echo "bench persistent rc=$rc"; cut -c1-600 gpurun_out/c2_pers.json; if [ $rc -ne 0 ]; then tail -20 gpurun_out/c2_pers.err; exit $rc; fi
timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu --persistent 0 > gpurun_out/c2_fork.json 2> gpurun_out/c2_fork.err
rc=$?; echo "bench forked rc=$rc"; cut -c1-400 gpurun_out/c2_fork.json; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2p -o run --output-format csv -- python bench.py --config c2 --steps 20 --warmup 5 --no-cpu --no-check > gpurun_out/prof_c2p.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find gpurun_out/prof_c2p -name "*kernel_stats.csv" -exec cat {} \; | grep swipes | cut -d, -f1-8
exit $rc
