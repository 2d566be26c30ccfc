#!/bin/bash
set -o pipefail
O=gpurun_out
mkdir -p $O/xdbg
timeout -k 10 200 python -u -m pytest tests/test_exchange_gpu.py -q -k route_cap --timeout 120 --timeout-method thread > $O/r04_routecap.log 2>&1; echo "route_cap tests rc=$?"; tail -15 $O/r04_routecap.log
EXCH_DEBUG=1 MASTER_ADDR=127.0.0.1 timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29711 tests/exchange_worker.py $O/xdbg async_overflow > $O/r04_xdbg.log 2>&1
echo "xdbg rc=$?"; grep -E "rank . (k1|route)|Error" $O/r04_xdbg.log | head -30
SKE_LIB=tools/ab/libsketch_al32fix.so timeout -k 10 120 python -u tools/diag_part.py 700333 2>&1 | grep -v amdgpu.ids > $O/diag_al32.log; echo "diag al32fix rc=$?"; cat $O/diag_al32.log
SKE_LIB=tools/ab/libsketch_al32fix.so timeout -k 10 200 python -u -m pytest tests/test_k1_partitioned.py -q --timeout 120 --timeout-method thread > $O/bis_al32fix.log 2>&1; echo "al32fix tests rc=$?"; tail -3 $O/bis_al32fix.log
timeout -k 10 200 python -u -m pytest tests/test_k1_partitioned.py -q --timeout 120 --timeout-method thread > $O/bis_tree.log 2>&1; echo "tree tests rc=$?"; tail -3 $O/bis_tree.log
for v in pc2 al32pc2; do SKE_LIB=tools/ab/libsketch_$v.so timeout -k 10 200 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/bis_$v.log 2>&1; echo "$v tests rc=$?"; tail -3 $O/bis_$v.log; done
LIBS="r03=tools/ab/libsketch_r03.so;tree=;a4nu=tools/ab/libsketch_a4nu.so;al32=tools/ab/libsketch_al32fix.so;al32nu=tools/ab/libsketch_al32nu.so;al32c2k=tools/ab/libsketch_al32c2k.so;al32split=tools/ab/libsketch_al32split.so;split=tools/ab/libsketch_split.so;pc2=tools/ab/libsketch_pc2.so;al32pc2=tools/ab/libsketch_al32pc2.so" ROUNDS=2 timeout -k 10 900 bash tools/ab_libs.sh > $O/r04_ab_libs2.txt 2>&1; echo "ab rc=$?"; cat $O/r04_ab_libs2.txt
timeout -k 10 300 bash tools/gpu_fetchcal.sh > $O/r04_fetchcal2.log 2>&1; echo "fetchcal rc=$?"; tail -3 $O/r04_fetchcal2.log
