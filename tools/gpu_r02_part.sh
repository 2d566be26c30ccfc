#!/bin/bash
# round 2: partitioned K1 -- parity tests, then C3 benches (sub-batch sizes) and a kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_k1_partitioned.py "tests/test_full_size.py::test_c3_gpu_shard_full_step" \
  "tests/test_full_size.py::test_c3_bench_shard_one_gpu" > gpurun_out/t_part.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_part.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/t_part.log; exit $rc; fi
for sub in 0 4194304 2097152; do
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu --streams 1 --graph 0 --part-sub $sub > gpurun_out/c3_part_$sub.json 2> gpurun_out/c3_part.err
rc=$?; echo "bench sub=$sub rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/c3_part_$sub.json'));print(d['value'],d['ms_per_step'])"
if [ $rc -ne 0 ]; then tail gpurun_out/c3_part.err; exit $rc; fi
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_part -o run --output-format csv -- python bench.py --config c3 --steps 20 --warmup 5 --no-cpu --streams 1 --graph 0 > gpurun_out/prof_part.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find gpurun_out/prof_part -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160 | head -6
exit $rc
