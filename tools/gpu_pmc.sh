#!/bin/bash
# GPU session: K1 ablations + PMC counter passes (one counter group per pass).
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
summ() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['k1_variant'])"; }
for a in 0 1 2 3 4; do
  for v in 1 0; do
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --ablate $a --variant $v > gpurun_out/abl.log 2>&1; rc=$?
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/abl.log; exit $rc; fi
    echo -n "ablate=$a variant=$v: "; summ gpurun_out/abl.log
  done
done
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
for c in FETCH_SIZE WRITE_SIZE "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "TCC_EA0_ATOMIC_sum" ; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc/$tag -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/pmc/$tag.log 2>&1; rc=$?
  echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$tag.log; fi
done
exit 0
