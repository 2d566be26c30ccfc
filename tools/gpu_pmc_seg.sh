#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only) over the
# default C3 bench (2^27 swipes per step, segmented PFADD); per-kernel
# summaries into gpurun_out/pmc_<ROUND>_<kernel>.json (tools/pmc_seg.py).
# usage: ROUND=r06 bash tools/gpu_pmc_seg.sh [extra bench args]
ARGS="--steps 4 --warmup 2 --no-cpu --no-check --secondary none --pass-replay 0 --host-fed 0 $*"
R=${ROUND:-r06}
mkdir -p gpurun_out/pmc_$R
export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum"
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum")
for c in "${GROUPS_[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/pmc_$R/$tag -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmc_$R/$tag.log 2>&1; rc=$?
  echo "pmc [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc_$R/$tag.log; exit $rc; fi
done
python tools/pmc_seg.py gpurun_out/pmc_$R gpurun_out/pmc_${R}_ || exit 1
