#!/bin/bash
# Build libsketch.so from the WORKING TREE with extra compile flags into
# tools/ab/libsketch_<name>.so (A/B of compile-time variants on one GPU box:
# SKE_LIB=tools/ab/libsketch_<name>.so python bench.py ...).
# usage: bash tools/ab_variant.sh <name> "-DSKE_PB_SPLIT=1 ..."
set -e
name=$1; extra=$2
root=$(git rev-parse --show-toplevel)
src="$root/tools/ab/src_$name"
rm -rf "$src"; mkdir -p "$src/real-time-student-attendance-system_amd"
cp -r "$root/include" "$src/"
cp -r "$root/real-time-student-attendance-system_amd/csrc" "$src/real-time-student-attendance-system_amd/"
rm -f "$src"/real-time-student-attendance-system_amd/csrc/*.o "$src"/real-time-student-attendance-system_amd/csrc/*.so
make -s -C "$src/real-time-student-attendance-system_amd/csrc" -j8 EXTRA="$extra" libsketch.so
cp "$src/real-time-student-attendance-system_amd/csrc/libsketch.so" "$root/tools/ab/libsketch_$name.so"
rm -rf "$src"
echo "tools/ab/libsketch_$name.so"
