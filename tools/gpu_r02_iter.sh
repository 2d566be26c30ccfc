#!/bin/bash
# round 2 iteration: partitioned K1 parity subset, C3 bench with pass timing, optional PMC
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_k1_partitioned.py "tests/test_full_size.py::test_c3_bench_shard_one_gpu" > gpurun_out/t_part.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_part.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/t_part.log; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_part -o run --output-format csv -- python bench.py --config c3 --steps 20 --warmup 5 --no-cpu --streams 1 --graph 0 > gpurun_out/prof_part.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof_part.log | cut -c1-300
find gpurun_out/prof_part -name "*kernel_stats.csv" -exec cat {} \; | grep part | cut -d, -f1-4
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$PMC" ]; then bash tools/gpu_pmc_part.sh; fi
