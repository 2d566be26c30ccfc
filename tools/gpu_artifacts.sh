#!/bin/bash
# Round artifacts for the default bench command: rocprofv3 kernel stats and
# PMC passes (separate runs, --pmc only), summarised for profiles/.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_art -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/prof_art.log 2>&1; rc=$?
echo "rocprof rc=$rc"; grep -m1 "k_swipes<0" gpurun_out/prof_art/run_kernel_stats.csv | cut -d, -f1,2,4,6,7 | cut -c1-40,150-
if [ $rc -ne 0 ]; then exit $rc; fi
TAG=c2 BENCH_ARGS="" bash tools/gpu_pmc.sh
