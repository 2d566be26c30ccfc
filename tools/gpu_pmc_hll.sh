#!/bin/bash
# A/B of the partitioned K1's PFADD forms at C3: hll_mode 0
# (pass C: pre-check load + CAS per raising register) against hll_mode 1
# (register-line ownership: partition by line, lines gathered into LDS,
# raised there, stored back whole).  Per form: kernel times (rocprofv3
# --kernel-trace --stats) and FETCH_SIZE / WRITE_SIZE / TCC_EA0_ATOMIC per
# dispatch of every PFADD kernel, one --pmc pass each.
#   usage: bash tools/gpu_pmc_hll.sh   -> gpurun_out/pmc_hll/
OUT=gpurun_out/pmc_hll
mkdir -p $OUT
export TMPDIR=/tmp
# the pre-cleanup library (round 3, commit of the launcher): the only build with hll_mode 1
export SKE_LIB=${SKE_LIB:-tools/ab/libsketch_r03.so}
ARGS="--config c3 --steps 20 --warmup 5 --no-cpu --no-check --secondary none --pass-replay 0"
for m in 0 1; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/stats_h$m -o run --output-format csv -- python bench.py $ARGS --opt hll_mode=$m > $OUT/stats_h$m.log 2>&1 || exit $?
  for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $c | tr ' ' '_')
    timeout -k 10 150 rocprofv3 --pmc $c -d $OUT/h$m/$tag -o run --output-format csv -- python bench.py $ARGS --opt hll_mode=$m > $OUT/h${m}_$tag.log 2>&1; rc=$?
    echo "hll_mode $m pmc [$c] rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
for k in k_part_a3 k_part_b k_part_c_fl; do python tools/pmc_summary.py $OUT/h0 $k $OUT/h0_$k.json 5 > /dev/null; done
for k in k_part_a2 k_part_b k_part_c2 k_part_hscan k_part_hd k_part_he; do python tools/pmc_summary.py $OUT/h1 $k $OUT/h1_$k.json 5 > /dev/null; done
echo "summaries written"
