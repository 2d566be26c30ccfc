#!/bin/bash
# round 2: the driver's bench command, then its rocprofv3 kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-1500 gpurun_out/bench_default.json
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_default.err; exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/prof_default.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find gpurun_out/prof_default -name "*kernel_stats.csv" -exec cat {} \; | grep -E "part|k_swipes" | cut -c1-150
exit $rc
