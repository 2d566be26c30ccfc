#!/bin/bash
# round 5 session w: where the world-1 exchange's 0.5 ms goes -- plain bench
# with fixed-width ids (the exchange's K1 form) and a kernel trace of --exchange 1
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0"
timeout -k 10 300 python -u bench.py $B --layout fixed > $O/r05w_fixed.json 2> $O/r05w_fixed.err || { echo "fixed failed"; tail -5 $O/r05w_fixed.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/r05w_fixed.json').read().strip().splitlines()[-1]); print('fixed', '%.4e'%d['value'], '%.3f ms/step'%d['ms_per_step'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r05w_trace -o run --output-format csv -- python bench.py $B --exchange 1 > $O/r05w_trace.log 2>&1 || { echo "trace failed"; tail -5 $O/r05w_trace.log; exit 1; }
f=$(find $O/r05w_trace -name "*kernel_stats.csv" | head -1); head -12 "$f"
