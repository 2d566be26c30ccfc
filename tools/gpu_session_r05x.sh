#!/bin/bash
# round 5 session x: can the probe records stay in the 256 MiB Infinity Cache
# between pass A and pass B?  Sub-batches of 16 M (704 MB of records), 4 M
# (176 MB) and 2 M (88 MB), with the records' nt policy (default build,
# SKE_NT 71) and without it (SKE_NT 3 build)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B --part-sub $PS > $O/r05x_$tag.json 2> $O/r05x_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05x_$tag.err; exit 1; }; }
for PS in 16777216 4194304 2097152; do
  run nt71_$PS SKE_NT_TAG=71
  run nt3_$PS SKE_LIB=tools/abv/libsketch_nt3.so
done
python tools/r05_passes.py $O/r05x_*.json
