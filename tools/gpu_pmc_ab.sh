#!/bin/bash
# PMC A/B of the two PFADD forms (CAS pass C vs the segmented PFADD): the
# bytes and atomics counters only, one group per rocprofv3 run.
# usage: bash tools/gpu_pmc_ab.sh <tag> [bench args]   -> gpurun_out/pmcab_<tag>/
TAG=$1; shift
ARGS="--steps 4 --warmup 2 --no-cpu --no-check --secondary none --pass-replay 0 --host-fed 0 $*"
mkdir -p gpurun_out/pmcab_$TAG
export TMPDIR=/tmp
GROUPS_=("WRITE_SIZE" "TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum")
for c in "${GROUPS_[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/pmcab_$TAG/$tag -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmcab_$TAG/$tag.log 2>&1; rc=$?
  echo "pmc $TAG [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmcab_$TAG/$tag.log; exit $rc; fi
done
