#!/bin/bash
# round 5 session aa: PMC passes of the new default (2^25 sub-batches), then
# the default bench line and its kernel trace
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
NSUB=4 STEP_SWIPES=134217728 bash tools/gpu_pmc_r05.sh || exit 1
mkdir -p $O/pmc_r05_out && cp $O/pmc_r05_*.json $O/pmc_r05_out/ 2>/dev/null
for k in k_part_a k_part_b k_part_c k_seg_d k_seg_e; do cp $O/pmc_r05_$k.json profiles/r05_pmc_c3_seg_$k.json; done
timeout -k 10 400 python -u bench.py > $O/r05aa_bench.json 2> $O/r05aa_bench.err || { echo "bench failed"; tail -5 $O/r05aa_bench.err; exit 1; }
python tools/r05_passes.py $O/r05aa_bench.json
python -c "
import json; d=json.loads(open('$O/r05aa_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print({k: r.get(k) for k in ('kernel','kernel_ms','achieved','frac','traffic','traffic_source')}); print(d['cpu_baseline'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r05aa_trace -o run --output-format csv -- python bench.py --no-cpu --secondary none --host-fed 0 > $O/r05aa_trace.log 2>&1 || { echo "trace failed"; tail -5 $O/r05aa_trace.log; exit 1; }
echo trace ok
