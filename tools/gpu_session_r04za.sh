#!/bin/bash
mkdir -p gpurun_out
# Round 4: region-ordered pass C (SKE_PC_REGIONS variant builds): parity of
# each variant on the partitioned-K1 tests, then an A/B against the base.
timeout -k 10 120 ./tools/regionbench > gpurun_out/r04_regionbench.json; echo "regionbench rc=$?"; cat gpurun_out/r04_regionbench.json
for v in reg13 reg7; do
  SKE_LIB=tools/ab/libsketch_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_k1_partitioned.py tests/test_full_size.py > gpurun_out/za_${v}_tests.log 2>&1
  rc=$?; echo "$v tests rc=$rc"; tail -2 gpurun_out/za_${v}_tests.log
  [ $rc -eq 0 ] || exit 1
done
LIBS="base=tools/ab/libsketch_base.so;reg13=tools/ab/libsketch_reg13.so;reg7=tools/ab/libsketch_reg7.so" ROUNDS=3 \
  bash tools/ab_libs.sh | tee gpurun_out/r04_ab_pc_regions.txt
