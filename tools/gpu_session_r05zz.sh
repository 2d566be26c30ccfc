#!/bin/bash
# round 5 session zz: E1 claiming per XCD (items i = b mod 8 from counter b mod 8)
# vs one counter; window pass bytes by PMC for both
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_seg_pfadd.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > $O/r05zz_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/r05zz_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05zz_$tag.json 2> $O/r05zz_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05zz_$tag.err; exit 1; }; }
for i in 1 2; do
  run new_$i X=1
  run base_$i SKE_LIB=tools/abv/libsketch_base.so
done
B="$B --shard 8"
run shnew X=1
run shbase SKE_LIB=tools/abv/libsketch_base.so
python tools/r05_passes.py $O/r05zz_*.json
ARGS="--steps 4 --warmup 2 --no-cpu --no-check --secondary none --pass-replay 0 --host-fed 0"
for v in new base; do
  L=""; [ $v = base ] && L=tools/abv/libsketch_base.so
  SKE_LIB=$L timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum -d $O/r05zz_pmc_$v -o run --output-format csv -- python bench.py $ARGS > $O/r05zz_pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
python tools/r05_pmc_kernels.py $O/r05zz_pmc.json "k_seg_e<1, false>" new=$O/r05zz_pmc_new base=$O/r05zz_pmc_base
