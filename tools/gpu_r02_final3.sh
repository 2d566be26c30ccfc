#!/bin/bash
# session-2 closing evidence: full -m gpu suite, smoke, the driver's bench
# command + its rocprofv3 kernel trace, per-pass PMC of the C3 partitioned K1,
# the C5 rollups, and a 2-rank (gloo) rehearsal of bench.py
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_r02_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_r02_bench.sh || exit $?
TAG=c3s2 BENCH_ARGS="--steps 20 --warmup 5 --no-check --no-cpu" bash tools/gpu_pmc_part.sh || exit $?
timeout -k 10 400 python tools/bench_rollup.py > gpurun_out/rollup_c5.json 2> gpurun_out/rollup_c5.err
rc=$?; echo "rollup rc=$rc"; tail -c 400 gpurun_out/rollup_c5.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/rollup_c5.err; exit $rc; fi
bash tools/gpu_r02_multi.sh
