#!/bin/bash
# Address / data path counters (TA, TD, TCP) of the partitioned K1's passes,
# one group per rocprofv3 --pmc run.   usage: TAG=c3ta bash tools/gpu_pmc_ta.sh
TAG=${TAG:-c3ta}
ARGS=${BENCH_ARGS:-"--config c3 --steps 6 --warmup 2 --no-cpu --secondary none --pass-replay 0 --streams 1 --graph 0"}
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
GROUPS_=("TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum GRBM_GUI_ACTIVE" "TD_TD_BUSY_sum TD_TC_STALL_sum"
 "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
 "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum")
for c in "${GROUPS_[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --pmc $c -d gpurun_out/pmc_$TAG/$tag -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmc_$TAG/$tag.log 2>&1; rc=$?
  echo "pmc [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc_$TAG/$tag.log; exit $rc; fi
done
for k in a b c; do
  python tools/pmc_summary.py gpurun_out/pmc_$TAG "k_part_$k" gpurun_out/pmc_${TAG}_$k.json 2 > /dev/null && echo "summary $k written"
done
