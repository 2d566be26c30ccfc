#!/bin/bash
# C3 (19.8 MB Bloom, XCD-partitioned K1): rocprofv3 kernel trace of the bench
# command, then FETCH_SIZE / WRITE_SIZE / L2 passes (one --pmc group per run),
# summarised per K1 invocation (hash + region + finish passes) into
# gpurun_out/pmc_c3.json.
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--config c3 --steps 20 --warmup 3 --no-cpu --secondary none --pass-replay 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python bench.py $ARGS > gpurun_out/prof_c3.log 2>&1; rc=$?
echo "rocprof c3 rc=$rc"; tail -1 gpurun_out/prof_c3.log | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_c3/$tag -o run --output-format csv -- python bench.py --config c3 --steps 8 --warmup 2 --no-cpu --secondary none --pass-replay 0 > gpurun_out/pmc_c3_$tag.log 2>&1; rc=$?
  echo "pmc [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc_c3_$tag.log; exit $rc; fi
done
python tools/pmc_summary.py --launch gpurun_out/pmc_c3 "k_xr_" gpurun_out/pmc_c3.json 2 > /dev/null && echo "summary written"
