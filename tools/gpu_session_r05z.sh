#!/bin/bash
# round 5 session z: C1 and D as full grids (one run / one chunk per block:
# a block's stores need not drain before the next unit's loads) vs the
# persistent 2-blocks-per-CU loops; two alternations
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0"
for i in 1 2; do
  for g in 0 1 2 3; do
    SKE_SEG_GRID=$g timeout -k 10 300 python -u bench.py $B > $O/r05z_g${g}_$i.json 2> $O/r05z_g${g}_$i.err || { echo "bench g$g failed"; tail -5 $O/r05z_g${g}_$i.err; exit 1; }
  done
done
python tools/r05_passes.py $O/r05z_g*.json
