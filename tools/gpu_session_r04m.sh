#!/bin/bash
# round 4 session m: final-build evidence -- default bench, kernel trace,
# per-pass PMC, and the config matrix (C1, C2, C4, C5, C3 x 200 steps, exchange)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py > $O/r04_bench6.json 2> $O/r04_bench6.err || { echo "bench failed"; tail -5 $O/r04_bench6.err; exit 1; }
echo "bench ok"; cut -c1-200 $O/r04_bench6.json
rm -rf $O/kt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --secondary none --no-cpu --no-check --pass-replay 0 > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
echo "trace ok"
rm -rf $O/pmc_r04c3f
TAG=r04c3f timeout -k 10 600 bash tools/gpu_pmc_part.sh > $O/r04_pmc_part2.log 2>&1 || { echo "pmc failed"; tail -5 $O/r04_pmc_part2.log; exit 1; }
echo "pmc ok"
SKIP_TESTS=1 SKIP_BENCH=1 MATRIX="--config c1;--config c2;--config c4;--config c5;--config c3 --steps 200;--exchange 1" timeout -k 10 900 bash tools/gpu_session.sh > $O/r04_matrix.txt 2>&1; rc=$?; echo "matrix rc=$rc"; cat $O/r04_matrix.txt | grep "^\["
