#!/bin/bash
# round 5 session cc: level-1 bucket count of the segmented PFADD (seg_b1 7 / 8
# (auto at C3) / 9) and window size (seg_klog 1 / 2) at the default step
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; timeout -k 10 300 python -u bench.py $B "$@" > $O/r05cc_$tag.json 2> $O/r05cc_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05cc_$tag.err; exit 1; }; }
for i in 1 2; do
  run b8_$i
  run b7_$i --opt seg_b1=7
  run b9_$i --opt seg_b1=9
done
run k2b8 --opt seg_klog=2
run k2b7 --opt seg_klog=2 --opt seg_b1=7
python tools/r05_passes.py $O/r05cc_*.json
