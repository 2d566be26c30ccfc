#!/bin/bash
# round 5 session h: window-pass stamps for 1- and 2-key windows at a 128M batch
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
for k in 1; do
timeout -k 10 300 python -u tools/stamps/run_seg_stamps.py --batch 134217728 --opt hll_seg=1 --opt seg_klog=$k > $O/r05h_b128m_k$k.json 2> $O/r05h_b128m_k$k.err || { echo "k$k failed"; tail -5 $O/r05h_b128m_k$k.err; exit 1; }
cut -c1-1500 $O/r05h_b128m_k$k.json
done
