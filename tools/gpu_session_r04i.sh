#!/bin/bash
# round 4 session i: full parity suite, smoke, self-launched gloo world 2
# (owner-routed and exchange input), exchange bench, default bench
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r04_gpu_tests4.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/r04_gpu_tests4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r04_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/r04_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > $O/r04_gloo2.json 2> $O/r04_gloo2.err || { echo "gloo2 failed"; tail -5 $O/r04_gloo2.err; exit 1; }
echo "gloo2 ok"; python -c "import json; d=json.loads(open('$O/r04_gloo2.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['check']['ok'], d.get('rank_shares', {}).get('rank_share_max'))"
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --exchange 1 --steps 3 --warmup 1 > $O/r04_gloo2x.json 2> $O/r04_gloo2x.err || { echo "gloo2 exchange failed"; tail -5 $O/r04_gloo2x.err; exit 1; }
echo "gloo2 exchange ok"; python -c "import json; d=json.loads(open('$O/r04_gloo2x.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['check']['ok'], d['check'].get('exchange', {}).get('ok'), d.get('exchange'))"
timeout -k 10 200 python -u bench.py --exchange 1 --secondary none --no-cpu > $O/r04_exch6.json 2> $O/r04_exch6.err || { echo "exch bench failed"; tail -5 $O/r04_exch6.err; exit 1; }
echo "exchange bench ok"; cut -c1-260 $O/r04_exch6.json
timeout -k 10 200 python -u bench.py > $O/r04_bench5.json 2> $O/r04_bench5.err || { echo "bench failed"; tail -5 $O/r04_bench5.err; exit 1; }
echo "bench ok"; cut -c1-260 $O/r04_bench5.json
