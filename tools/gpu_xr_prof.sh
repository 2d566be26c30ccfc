#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xr -o run --output-format csv -- python bench.py --config c3 --steps 12 --warmup 3 --no-cpu > gpurun_out/prof_xr.log 2>&1; echo "rc=$?"
python -c "import csv; [print(r[\"Name\"][:40], r[\"Calls\"], r[\"AverageNs\"], r[\"MinNs\"]) for r in csv.DictReader(open(\"gpurun_out/prof_xr/run_kernel_stats.csv\")) if \"xr\" in r[\"Name\"] or \"k_swipes\" in r[\"Name\"]]"
for c in "TCC_HIT_sum TCC_MISS_sum" FETCH_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_xr/$tag -o run --output-format csv -- python bench.py --config c3 --steps 8 --warmup 2 --no-cpu > gpurun_out/pmc_xr_$tag.log 2>&1; echo "pmc $c rc=$?"
done
python tools/pmc_summary.py gpurun_out/pmc_xr "k_xr_region" gpurun_out/pmc_xr_probe.json 2 > /dev/null
python tools/pmc_summary.py gpurun_out/pmc_xr "k_xr_finish" gpurun_out/pmc_xr_finish.json 2 > /dev/null; python tools/pmc_summary.py gpurun_out/pmc_xr "k_xr_hash" gpurun_out/pmc_xr_hash.json 2 > /dev/null
echo done
