#!/bin/bash
# round 5 session y: sub-batches of up to 32M swipes (the per-sub-batch fixed
# costs -- pass B's image restaging, the segmented PFADD's per-sub-batch
# kernels -- amortised over twice the swipes); parity tests, then A/B 32M
# (default) vs 16M, two alternations
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_seg_pfadd.py tests/test_k1_partitioned.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > $O/r05y_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/r05y_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B > $O/r05y_s32_$i.json 2> $O/r05y_s32_$i.err || { echo "bench s32 failed"; tail -5 $O/r05y_s32_$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py $B --part-sub 16777216 > $O/r05y_s16_$i.json 2> $O/r05y_s16_$i.err || { echo "bench s16 failed"; tail -5 $O/r05y_s16_$i.err; exit 1; }
done
python tools/r05_passes.py $O/r05y_s*.json
