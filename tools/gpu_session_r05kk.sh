#!/bin/bash
# round 5 session kk: window size on the late tree (seg_klog 1 default vs 0),
# N = 1 and the 8-way shard
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; timeout -k 10 300 python -u bench.py $B "$@" > $O/r05kk_$tag.json 2> $O/r05kk_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05kk_$tag.err; exit 1; }; }
for i in 1 2; do
  run k1_$i
  run k0_$i --opt seg_klog=0
done
run s8k1 --shard 8
run s8k0 --shard 8 --opt seg_klog=0
python tools/r05_passes.py $O/r05kk_*.json
