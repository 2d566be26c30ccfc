#!/bin/bash
# session-2 final check: full -m gpu suite, smoke, the driver's bench command +
# its rocprofv3 kernel trace, the C5 rollups and the PCIe-inclusive host feed
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_r02_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_r02_bench.sh || exit $?
timeout -k 10 400 python tools/bench_rollup.py > gpurun_out/rollup_c5.json 2> gpurun_out/rollup_c5.err
rc=$?; echo "rollup rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/rollup_c5.err; exit $rc; fi
timeout -k 10 300 python tools/bench_host_feed.py > gpurun_out/host_feed.json 2> gpurun_out/host_feed.err
rc=$?; echo "host feed rc=$rc"; exit $rc
