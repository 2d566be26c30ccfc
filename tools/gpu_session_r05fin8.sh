#!/bin/bash
# round 5 session fin8 (rerun of o on the final tree): the driver's 8-GPU command shape rehearsed on one GPU
# (gloo, 8 ranks on the card), owner-routed and through the exchange; C5's
# rollup queries at world 2 (gloo)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 600 python -u bench.py --gpus 8 --dist-backend gloo --steps 3 --warmup 1 > $O/r05fin8_gloo8.json 2> $O/r05fin8_gloo8.err || { echo "gloo8 failed"; tail -8 $O/r05fin8_gloo8.err; exit 1; }
t1=$(date +%s); echo "gloo8 owner-routed wall $((t1-t0)) s"
python -c "import json; d=json.loads(open('$O/r05fin8_gloo8.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['check']['ok'], d['check'].get('exchange',{}).get('ok'), d['rank_shares']['slowest_rank'], d['roofline'].get('passes_of_rank'), [round(x,1) for x in d['rank_shares']['device_mem_used_GB']])"
timeout -k 10 600 python -u bench.py --gpus 8 --dist-backend gloo --exchange 1 --steps 3 --warmup 1 > $O/r05fin8_gloo8x.json 2> $O/r05fin8_gloo8x.err || { echo "gloo8 exchange failed"; tail -8 $O/r05fin8_gloo8x.err; exit 1; }
t2=$(date +%s); echo "gloo8 exchange wall $((t2-t1)) s"
python -c "import json; d=json.loads(open('$O/r05fin8_gloo8x.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['check']['ok'], d.get('exchange'))"
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --config c5 --steps 3 --warmup 1 > $O/r05fin8_c5_gloo2.json 2> $O/r05fin8_c5_gloo2.err || { echo "c5 gloo2 failed"; tail -8 $O/r05fin8_c5_gloo2.err; exit 1; }
t3=$(date +%s); echo "c5 gloo2 wall $((t3-t2)) s"
python -c "import json; d=json.loads(open('$O/r05fin8_c5_gloo2.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['check']['ok'], json.dumps(d.get('rollup'))[:500])"
