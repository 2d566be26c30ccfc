#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only) over the
# default bench; summary of K1 into gpurun_out/pmc_<tag>.json.
# usage: TAG=r01 BENCH_ARGS="..." KERNEL="k_swipes_lds<true" bash tools/gpu_pmc.sh
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS"
 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" "SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT")
for c in "${GROUPS_[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_$TAG/$tag -o run --output-format csv -- python bench.py --steps 12 --warmup 3 --no-cpu --secondary none --pass-replay 0 $BENCH_ARGS > gpurun_out/pmc_$TAG/$tag.log 2>&1; rc=$?
  echo "pmc [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc_$TAG/$tag.log; exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmc_$TAG "${KERNEL:-k_swipes_lds<true}" gpurun_out/pmc_$TAG.json 3 > /dev/null && echo "summary written"
