#!/bin/bash
# Build diagnostic variants of the in-tree libsketch with extra -D flags into
# tools/ab/libsketch_<name>.so (A/B: SKE_LIB=tools/ab/libsketch_<name>.so).
# usage: bash tools/ab_variants.sh name1 "-DFLAG=1" [name2 "-DFLAG=2" ...]
set -e
root=$(git rev-parse --show-toplevel)
mkdir -p "$root/tools/ab"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  tmp=$(mktemp -d)
  mkdir -p "$tmp/pkg" "$tmp/include"
  cp -r "$root/real-time-student-attendance-system_amd/csrc" "$tmp/pkg/csrc"
  cp "$root/include/sketch.h" "$tmp/include/"
  (cd "$tmp/pkg/csrc" && rm -f *.o libsketch.so && make -s -j8 FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $defs" libsketch.so)
  cp "$tmp/pkg/csrc/libsketch.so" "$root/tools/ab/libsketch_$name.so"
  rm -rf "$tmp"
  echo "tools/ab/libsketch_$name.so ($defs)"
done
