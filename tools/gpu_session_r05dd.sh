#!/bin/bash
# round 5 session dd: level-1 buckets at the 8-way shard (12.5 k keys: auto b1 6)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0 --shard 8"
run() { tag=$1; shift; timeout -k 10 300 python -u bench.py $B "$@" > $O/r05dd_$tag.json 2> $O/r05dd_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05dd_$tag.err; exit 1; }; }
for i in 1 2; do
  run b6_$i
  run b5_$i --opt seg_b1=5
  run b4_$i --opt seg_b1=4
done
python tools/r05_passes.py $O/r05dd_*.json
