#!/bin/bash
# PMC passes over the C2 bench's persistent LDS K1 (one counter group per
# rocprofv3 run, --pmc only); summaries to gpurun_out/pmc_<TAG>.json.
# usage: TAG=c2p BENCH_ARGS="--config c2 --steps 20 --warmup 5" bash tools/gpu_pmc_c2.sh
TAG=${TAG:-c2p}
ARGS=${BENCH_ARGS:-"--config c2 --steps 20 --warmup 5"}
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS"
 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" "SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT")
for c in "${GROUPS_[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --pmc $c -d gpurun_out/pmc_$TAG/$tag -o run --output-format csv -- python bench.py $ARGS --no-cpu --secondary none --pass-replay 0 --no-check > gpurun_out/pmc_$TAG/$tag.log 2>&1; rc=$?
  echo "pmc [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc_$TAG/$tag.log; exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmc_$TAG "k_swipes_lds_many" gpurun_out/pmc_${TAG}.json 1 > /dev/null && echo "summary written"
