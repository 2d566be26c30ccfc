#!/bin/bash
# round 2 closing evidence: smoke, the driver's default bench (C3) + rocprofv3
# kernel trace, per-pass PMC of C3, the C2 bench + rocprofv3 + PMC
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_r02_bench.sh || exit $?
TAG=c3 BENCH_ARGS="--steps 20 --warmup 5 --no-check" bash tools/gpu_pmc_part.sh || exit $?
timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err; rc=$?
echo "bench c2 rc=$rc"; cut -c1-300 gpurun_out/bench_c2.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_c2.err; exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --config c2 --steps 20 --warmup 5 --no-cpu > gpurun_out/prof_c2.log 2>&1; rc=$?
echo "rocprof c2 rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_c2.log; exit $rc; fi
TAG=c2p20 BENCH_ARGS="--config c2 --steps 20 --warmup 5" bash tools/gpu_pmc_c2.sh
