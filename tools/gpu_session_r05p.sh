#!/bin/bash
# round 5 session p: PMC A/B of the PFADD forms at N=1 (2^27 swipes) and at the 8-way shard
set -o pipefail
bash tools/gpu_pmc_ab.sh cas_n1 --opt hll_seg=0 || exit 1
bash tools/gpu_pmc_ab.sh seg_shard8 --shard 8 || exit 1
bash tools/gpu_pmc_ab.sh cas_shard8 --shard 8 --opt hll_seg=0 || exit 1
bash tools/gpu_pmc_ab.sh seg_shard8_16m --shard 8 --batch 16000000 --opt hll_seg=1 || exit 1
bash tools/gpu_pmc_ab.sh cas_shard8_16m --shard 8 --batch 16000000 --opt hll_seg=0 || exit 1
