#!/bin/bash
# round 5 session u: why the pipelined exchange does not overlap -- stream
# layouts (4 streams / return half on K1's stream / routing at high
# priority) and hardware queues (GPU_MAX_HW_QUEUES 4 vs 8)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
B="--no-cpu --secondary none --host-fed 0 --exchange 1"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py $B > $O/r05u_$tag.json 2> $O/r05u_$tag.err || { echo "bench $tag failed"; tail -5 $O/r05u_$tag.err; exit 1; }; }
run s4 SKE_XPIPE=
run s3 SKE_XPIPE=3
run s3p SKE_XPIPE=3p
run s4q8 SKE_XPIPE= GPU_MAX_HW_QUEUES=8
run s3q8 SKE_XPIPE=3 GPU_MAX_HW_QUEUES=8
run s3pq8 SKE_XPIPE=3p GPU_MAX_HW_QUEUES=8
for f in $O/r05u_*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], '%.4e'%d['value'], '%.3f ms/step'%d['ms_per_step'], d['check']['ok'])"; done
