#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only) over the C3
# bench; per-kernel summaries of the partitioned K1's passes into
# gpurun_out/pmc_<TAG>_{a,b,c}.json.   usage: TAG=c3 bash tools/gpu_pmc_part.sh
TAG=${TAG:-c3}
# the bench's own steps (20 timed after 5 warm-up; the summaries skip the
# warm-up dispatches), so per-dispatch counters describe the timed steps
ARGS=${BENCH_ARGS:-"--config c3 --steps 20 --warmup 5 --no-cpu --no-check --secondary none --pass-replay 0 --streams 1 --graph 0"}
SKIP=${SKIP:-5}
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS"
 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" "SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT")
for c in "${GROUPS_[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --pmc $c -d gpurun_out/pmc_$TAG/$tag -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmc_$TAG/$tag.log 2>&1; rc=$?
  echo "pmc [$c] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc_$TAG/$tag.log; exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmc_$TAG "k_part_a" gpurun_out/pmc_${TAG}_a.json $SKIP > /dev/null && echo "summary a written"
# every read request is counted by size (hbm_bytes_calibrated, tools/fetchcal.hip)
python tools/pmc_summary.py gpurun_out/pmc_$TAG "k_part_b" gpurun_out/pmc_${TAG}_b.json $SKIP > /dev/null && echo "summary b written"
python tools/pmc_summary.py gpurun_out/pmc_$TAG "k_part_c" gpurun_out/pmc_${TAG}_c.json $SKIP > /dev/null && echo "summary c written"
