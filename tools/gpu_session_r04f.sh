#!/bin/bash
# round 4 session f: wave-aggregated routing ranks (exchange tests, --exchange 1
# bench + kernel trace), C2 PMC passes, the default bench.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_exchange_gpu.py tests/test_k1_partitioned.py -q --timeout 120 --timeout-method thread > $O/f_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --exchange 1 --secondary none --no-cpu > $O/r04_exch3.json 2> $O/r04_exch3.err || { echo "exch bench failed"; tail -5 $O/r04_exch3.err; exit 1; }
echo "exchange bench ok"; cut -c1-300 $O/r04_exch3.json
rm -rf $O/ktx
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ktx -o run --output-format csv -- python bench.py --exchange 1 --secondary none --no-cpu --no-check --pass-replay 0 > $O/ktx.log 2>&1 || { echo "ktx failed"; tail -5 $O/ktx.log; exit 1; }
echo "kernel trace (exchange) ok"
rm -rf $O/pmc_r04c2
TAG=r04c2 timeout -k 10 600 bash tools/gpu_pmc_c2.sh > $O/r04_pmc_c2.log 2>&1 || { echo "pmc c2 failed"; tail -5 $O/r04_pmc_c2.log; exit 1; }
echo "pmc c2 ok"
timeout -k 10 200 python -u bench.py > $O/r04_bench3.json 2> $O/r04_bench3.err || { echo "bench failed"; tail -5 $O/r04_bench3.err; exit 1; }
echo "bench ok"; cut -c1-300 $O/r04_bench3.json
SKE_LIB=tools/ab/libsketch_pbx.so timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -q --timeout 120 --timeout-method thread > $O/f_pbx.log 2>&1; rc=$?; echo "pbx tests rc=$rc"; tail -3 $O/f_pbx.log; [ $rc -eq 0 ] || exit $rc
LIBS="tree=;pbx=tools/ab/libsketch_pbx.so" ROUNDS=3 timeout -k 10 400 bash tools/ab_libs.sh > $O/r04_ab_pbx.txt 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/r04_ab_pbx.txt
for v in tree pbx; do
  if [ $v = pbx ]; then export SKE_LIB=tools/ab/libsketch_pbx.so; else unset SKE_LIB; fi
  rm -rf $O/pmcb_$v
  timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_HIT_sum TCC_MISS_sum -d $O/pmcb_$v -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-check --secondary none --pass-replay 0 > $O/pmcb_$v.log 2>&1 || { echo "pmcb $v failed"; tail -3 $O/pmcb_$v.log; exit 1; }
  python tools/pmc_summary.py $O/pmcb_$v k_part_b $O/pmcb_$v.json 5 > /dev/null && python -c "import json; m=json.load(open('$O/pmcb_$v.json'))['mean']; print('$v', {k: round(v/1e6, 3) for k, v in m.items()})"
done
unset SKE_LIB
