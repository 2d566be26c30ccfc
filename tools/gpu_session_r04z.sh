#!/bin/bash
# Round 4: pass A at three blocks per CU (SKE_PA_BPC=3: 80 VGPRs, 56 B/lane
# of spills) -- parity of the variant, then an A/B against the base build.
mkdir -p gpurun_out
SKE_LIB=tools/ab/libsketch_bpc3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_k1_partitioned.py tests/test_full_size.py > gpurun_out/z_bpc3_tests.log 2>&1
echo "bpc3 tests rc=$?"; tail -2 gpurun_out/z_bpc3_tests.log
LIBS="base=tools/ab/libsketch_base.so;bpc3=tools/ab/libsketch_bpc3.so" ROUNDS=3 bash tools/ab_libs.sh | tee gpurun_out/r04_ab_pa_bpc3.txt
