#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only) over the C3
# bench; per-kernel summaries of the partitioned K1's passes into
# gpurun_out/pmc_<TAG>_{a,b,c}.json.   usage: TAG=c3 bash tools/gpu_pmc_part.sh
TAG=${TAG:-c3}
ARGS=${BENCH_ARGS:-"--config c3 --steps 8 --warmup 2 --no-cpu --secondary none --pass-replay 0 --streams 1 --graph 0"}
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS"
 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" "SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT")
for c in "${GROUPS_[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --pmc $c -d gpurun_out/pmc_$TAG/$tag -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmc_$TAG/$tag.log 2>&1; rc=$?
  echo "pmc [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc_$TAG/$tag.log; exit $rc; fi
done
for k in a b c; do
  python tools/pmc_summary.py gpurun_out/pmc_$TAG "k_part_$k" gpurun_out/pmc_${TAG}_$k.json 2 > /dev/null && echo "summary $k written"
done
