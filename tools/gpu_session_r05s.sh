#!/bin/bash
# round 5 session s: PMC bytes of passes A and B, per-tile runs vs the group layout
set -o pipefail
bash tools/gpu_pmc_ab.sh rg0 --opt rec_groups=0 || exit 1
bash tools/gpu_pmc_ab.sh rg1 --opt rec_groups=1 || exit 1
python tools/r05_pmc_kernels.py gpurun_out/r05s_pmc_rec_groups.json k_part_a3,k_part_b rg0=gpurun_out/pmcab_rg0 rg1=gpurun_out/pmcab_rg1
