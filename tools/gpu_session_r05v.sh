#!/bin/bash
# round 5 session v: the exchange at world 1 as the identity (slots mapped,
# K1 in place); exchange tests; bench N=1 plain vs --exchange 1, two alternations
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_exchange_gpu.py -k "solo or async" -x -q --timeout 200 --timeout-method thread > $O/r05v_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/r05v_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu --secondary none --host-fed 0"
for i in 1 2; do
  for x in 0 1; do
    timeout -k 10 300 python -u bench.py $B --exchange $x > $O/r05v_x${x}_$i.json 2> $O/r05v_x${x}_$i.err || { echo "bench x$x failed"; tail -5 $O/r05v_x${x}_$i.err; exit 1; }
  done
done
for f in $O/r05v_x*_*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], '%.4e'%d['value'], '%.3f ms/step'%d['ms_per_step'], 'enqueue_us', round(d.get('host_enqueue_us_per_step',0),1), d['check']['ok'], json.dumps(d.get('exchange'))[:160])"; done
