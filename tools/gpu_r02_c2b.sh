#!/bin/bash
# C2 persistent K1: tile sweep under rocprof
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 1 2 4; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2t$t -o run --output-format csv -- python bench.py --config c2 --steps 20 --warmup 5 --no-cpu --no-check --tile $t > gpurun_out/c2t$t.json 2>gpurun_out/c2t$t.err
rc=$?; echo "tile $t rc=$rc"; cut -c1-330 gpurun_out/c2t$t.json
find gpurun_out/prof_c2t$t -name "*kernel_stats.csv" -exec cat {} \; | grep swipes_lds | cut -d, -f1-5
if [ $rc -ne 0 ]; then tail -5 gpurun_out/c2t$t.err; exit $rc; fi
done
