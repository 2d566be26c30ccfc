#!/bin/bash
# round-4 GPU session b: diagnostics of the line-aligned pass A and of the
# exchange overflow re-run, then parity suite, bench, A/B of builds, exchange
# benches, FETCH_SIZE calibration, hll_mode A/B.
set -o pipefail
O=gpurun_out
mkdir -p $O/xdbg
SKE_LIB=tools/ab/libsketch_al32fix.so timeout -k 10 120 python -u tools/diag_part.py 700333 2>&1 | grep -v amdgpu.ids > $O/diag_al32.log; echo "diag al32fix rc=$?"; cat $O/diag_al32.log
SKE_LIB=tools/ab/libsketch_al32fix.so timeout -k 10 200 python -u -m pytest tests/test_k1_partitioned.py -q --timeout 120 --timeout-method thread > $O/bis_al32fix.log 2>&1; echo "al32fix tests rc=$?"; tail -3 $O/bis_al32fix.log
EXCH_DEBUG=1 MASTER_ADDR=127.0.0.1 timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29711 tests/exchange_worker.py $O/xdbg async_overflow > $O/r04_xdbg.log 2>&1
echo "xdbg rc=$?"; grep -E "rank . k1|Error|error" $O/r04_xdbg.log | head -20
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  --deselect "tests/test_exchange_gpu.py::test_exchange_on_device_equals_oracle[2-async_overflow]" > $O/r04_gpu_tests.log 2>&1; echo "gpu tests rc=$?"; tail -12 $O/r04_gpu_tests.log
timeout -k 10 200 python -u bench.py > $O/r04_bench1.json 2> $O/r04_bench1.err || exit 1
echo "bench ok"
LIBS="r03=tools/ab/libsketch_r03.so;tree=;split=tools/ab/libsketch_split.so;al32=tools/ab/libsketch_al32fix.so;al32split=tools/ab/libsketch_al32split.so" ROUNDS=2 timeout -k 10 500 bash tools/ab_libs.sh > $O/r04_ab_libs.txt 2>&1 || { cat $O/r04_ab_libs.txt; exit 1; }
cat $O/r04_ab_libs.txt
timeout -k 10 200 python -u bench.py --exchange 1 --secondary none --no-cpu > $O/r04_exch1.json 2> $O/r04_exch1.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --exchange 1 --steps 3 --warmup 1 > $O/r04_exch_gloo2.json 2> $O/r04_exch_gloo2.err || exit 1
echo "exchange benches ok"
timeout -k 10 300 bash tools/gpu_fetchcal.sh > $O/r04_fetchcal.log 2>&1 || { tail -5 $O/r04_fetchcal.log; exit 1; }
echo "fetchcal ok"
timeout -k 10 600 bash tools/gpu_pmc_hll.sh > $O/r04_pmc_hll.log 2>&1 || { tail -5 $O/r04_pmc_hll.log; exit 1; }
echo "pmc hll ok"
