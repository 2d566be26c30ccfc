#!/bin/bash
# FETCH_SIZE calibration (tools/fetchcal.hip): the list of counters this box
# offers, then one rocprofv3 --pmc pass per counter group over fetchcal, and
# the per-kernel summary (tools/fetchcal_summary.py).
#   usage: bash tools/gpu_fetchcal.sh   (fetchcal built beforehand, in-tree)
set -o pipefail
OUT=gpurun_out/fetchcal
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
timeout -k 10 120 ./tools/fetchcal > $OUT/times.json || exit $?
GROUPS_=("FETCH_SIZE" "TCC_MISS_sum TCC_HIT_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_REQ_sum" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_SECTORS_sum")
for c in "${GROUPS_[@]}"; do
  ok=1
  for x in $c; do grep -q "${x%_sum}" $OUT/avail.txt || { echo "skip [$c]: $x not offered"; ok=0; }; done
  [ $ok = 1 ] || continue
  tag=$(echo $c | tr ' ' '_')
  timeout -s KILL 60 rocprofv3 --pmc $c -d $OUT/$tag -o run --output-format csv -- ./tools/fetchcal > $OUT/$tag.log 2>&1; rc=$?
  echo "pmc [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $OUT/$tag.log; exit $rc; fi
done
python tools/fetchcal_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
