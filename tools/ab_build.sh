#!/bin/bash
# Build libsketch.so from a git revision into tools/ab/libsketch_<name>.so for
# A/B timing on one GPU box:  SKE_LIB=tools/ab/libsketch_base.so python bench.py
# usage: bash tools/ab_build.sh <rev> <name>
set -e
rev=$1; name=$2
root=$(git rev-parse --show-toplevel)
tmp="$root/tools/ab/src_$name"
rm -rf "$tmp"; mkdir -p "$tmp"
git -C "$root" archive "$rev" real-time-student-attendance-system_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/real-time-student-attendance-system_amd/csrc" -j8 libsketch.so
mkdir -p "$root/tools/ab"
cp "$tmp/real-time-student-attendance-system_amd/csrc/libsketch.so" "$root/tools/ab/libsketch_$name.so"
rm -rf "$tmp"
echo "tools/ab/libsketch_$name.so"
