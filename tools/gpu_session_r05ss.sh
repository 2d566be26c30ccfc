#!/bin/bash
# round 5 session ss: records per thread per round of the window pass at klog 1
# (4 default; 8 spills 84 B; 2 none)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05ss_$tag.json 2> $O/r05ss_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05ss_$tag.err; exit 1; }; }
for i in 1 2; do
  run r4_$i X=1
  run r8_$i SKE_LIB=tools/abv/libsketch_rpt8.so
  run r2_$i SKE_LIB=tools/abv/libsketch_rpt2.so
done
python tools/r05_passes.py $O/r05ss_*.json
