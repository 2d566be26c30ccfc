#!/bin/bash
# Instruction-mix PMC passes (one counter group per rocprofv3 run) over the
# bench; summary of the short-id LDS K1 into gpurun_out/pmci_<tag>.json.
# usage: TAG=c2 BENCH_ARGS="..." bash tools/gpu_pmc_insts.sh
mkdir -p gpurun_out/pmci_$TAG
export TMPDIR=/tmp
GROUPS_=("SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES"
 "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VSKIPPED GRBM_GUI_ACTIVE GRBM_COUNT")
for c in "${GROUPS_[@]}"; do
  tag=$(echo $c | tr ' ' '_' | cut -c1-60)
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmci_$TAG/$tag -o run --output-format csv -- python bench.py --steps 12 --warmup 3 --no-cpu --secondary none --pass-replay 0 $BENCH_ARGS > gpurun_out/pmci_$TAG/$tag.log 2>&1; rc=$?
  echo "pmc [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmci_$TAG/$tag.log; exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmci_$TAG "${KERNEL:-k_swipes_lds<true}" gpurun_out/pmci_$TAG.json 3 > /dev/null && echo "summary written"
