#!/bin/bash
# round 2 evidence for profiles/: the driver's default bench command (C3), its
# rocprofv3 kernel trace, the PMC passes of the three partitioned passes, the
# random-access and run-read microbenchmarks.
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_r02_bench.sh || exit $?
TAG=c3 BENCH_ARGS="--steps 20 --warmup 5 --no-check" bash tools/gpu_pmc_part.sh || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --config c2 --steps 20 --warmup 5 --no-cpu > gpurun_out/prof_c2.log 2>&1; rc=$?
echo "rocprof c2 rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_c2.log; exit $rc; fi
timeout -k 10 120 ./tools/randbench > gpurun_out/randbench.json 2> gpurun_out/randbench.err; rc=$?
echo "randbench rc=$rc"; cat gpurun_out/randbench.json | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 ./tools/runbench > gpurun_out/runbench.json 2> gpurun_out/runbench.err; rc=$?
echo "runbench rc=$rc"; cat gpurun_out/runbench.json | cut -c1-400; exit $rc
