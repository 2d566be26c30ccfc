#!/bin/bash
# round 5 session r: where the group layout's pass A time goes -- the layout
# (g1), every run in its tile's overflow row (g1 + SKE_GL_DIAG: same compute,
# contiguous writes), the layout without nt on the copy-out (SKE_NT=3 build),
# the per-tile layout (g0); two alternations
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B --opt rec_groups=0 > $O/r05r_g0_$i.json 2> $O/r05r_g0_$i.err || { echo "g0 failed"; tail -5 $O/r05r_g0_$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py $B --opt rec_groups=1 > $O/r05r_g1_$i.json 2> $O/r05r_g1_$i.err || { echo "g1 failed"; tail -5 $O/r05r_g1_$i.err; exit 1; }
  SKE_GL_DIAG=1 timeout -k 10 300 python -u bench.py $B --opt rec_groups=1 > $O/r05r_g1diag_$i.json 2> $O/r05r_g1diag_$i.err || { echo "g1diag failed"; tail -5 $O/r05r_g1diag_$i.err; exit 1; }
  SKE_LIB=tools/abl/libsketch_nt3.so timeout -k 10 300 python -u bench.py $B --opt rec_groups=1 > $O/r05r_g1nt3_$i.json 2> $O/r05r_g1nt3_$i.err || { echo "g1nt3 failed"; tail -5 $O/r05r_g1nt3_$i.err; exit 1; }
done
python tools/r05_passes.py $O/r05r_*.json
