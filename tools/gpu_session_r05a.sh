#!/bin/bash
# round 5 session a: pass times of the shipped K1 at the 8-way C3 shard and at
# larger N=1 batches (the regimes of the segmented HLL form)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --secondary none "$@" > $O/r05a_$n.json 2> $O/r05a_$n.err || { echo "$n failed"; tail -5 $O/r05a_$n.err; exit 1; }
  python tools/r05_passes.py $O/r05a_$n.json
}
run base
run shard8 --shard 8
run b64m --batch 67108864 --steps 6 --warmup 2
run b128m --batch 134217728 --steps 4 --warmup 2
run shard8_b64m --shard 8 --batch 67108864 --steps 6 --warmup 2
