#!/bin/bash
# Round 4: the non-temporal policy bits on the final build (SKE_NT 7 default;
# 15 adds pass A's HLL words and fail bytes, 23 pass C's streams) -- A/B only
# (the policy changes no result).
mkdir -p gpurun_out
LIBS="base=tools/ab/libsketch_base.so;nt15=tools/ab/libsketch_nt15.so;nt23=tools/ab/libsketch_nt23.so" ROUNDS=3 \
  bash tools/ab_libs.sh | tee gpurun_out/r04_ab_nt.txt
