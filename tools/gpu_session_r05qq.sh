#!/bin/bash
# round 5 session qq: 64 k-record slices (klog 1) at the 8-way shard
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0 --shard 8"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05qq_$tag.json 2> $O/r05qq_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05qq_$tag.err; exit 1; }; }
for i in 1 2; do
  run s32k_$i X=1
  run s64k_$i SKE_LIB=tools/abv/libsketch_slice32768.so
done
python tools/r05_passes.py $O/r05qq_*.json
