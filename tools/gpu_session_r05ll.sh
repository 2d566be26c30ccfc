#!/bin/bash
# round 5 session ll: PMC passes, the default bench line and its kernel trace
# on the final round-5 kernels
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
rm -rf $O/pmc_r05 $O/pmc_r05_*.json
NSUB=4 STEP_SWIPES=134217728 bash tools/gpu_pmc_r05.sh || exit 1
timeout -k 10 400 python -u bench.py > $O/r05ll_bench.json 2> $O/r05ll_bench.err || { echo "bench failed"; tail -5 $O/r05ll_bench.err; exit 1; }
python tools/r05_passes.py $O/r05ll_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r05ll_trace -o run --output-format csv -- python bench.py --no-cpu --secondary none --host-fed 0 > $O/r05ll_trace.log 2>&1 || { echo "trace failed"; tail -5 $O/r05ll_trace.log; exit 1; }
echo trace ok
