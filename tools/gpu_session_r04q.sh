#!/bin/bash
# round 4 session q: what pass B's image restaging costs (diagnostic build that
# stages a block's first unit only; answers wrong, times only)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
LIBS="tree=;nofail=tools/ab/libsketch_nofail.so;onestagenf=tools/ab/libsketch_onestagenf.so" ROUNDS=3 timeout -k 10 400 bash tools/ab_libs.sh > $O/r04_ab_restage.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_restage.txt
