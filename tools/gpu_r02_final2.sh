#!/bin/bash
# closing evidence after the pass-A change: full -m gpu suite, smoke, driver bench + rocprof, C3 PMC
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_r02_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_r02_bench.sh || exit $?
TAG=c3 BENCH_ARGS="--steps 20 --warmup 5 --no-check" bash tools/gpu_pmc_part.sh
