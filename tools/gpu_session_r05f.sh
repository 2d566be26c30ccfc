#!/bin/bash
# round 5 session f: window-pass stamps (diagnostic build) at the shard and a 128M batch
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/stamps/run_seg_stamps.py --shard 8 --opt hll_seg=1 --opt seg_klog=2 > $O/r05f_shard.json 2> $O/r05f_shard.err || { echo "shard failed"; tail -5 $O/r05f_shard.err; exit 1; }
cat $O/r05f_shard.json
timeout -k 10 300 python -u tools/stamps/run_seg_stamps.py --batch 134217728 --opt hll_seg=1 --opt seg_klog=2 > $O/r05f_b128m.json 2> $O/r05f_b128m.err || { echo "b128m failed"; tail -5 $O/r05f_b128m.err; exit 1; }
cat $O/r05f_b128m.json
