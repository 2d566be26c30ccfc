#!/bin/bash
# round 4 session zd: four self-launched ranks on one GPU (gloo), owner-routed
# and through the exchange -- the N = 4 code path of the driver's scaling run
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 4 --dist-backend gloo --steps 3 --warmup 1 --no-cpu > $O/r04_selflaunch_gloo4.json 2> $O/r04_selflaunch_gloo4.err || { echo "gloo4 failed"; tail -5 $O/r04_selflaunch_gloo4.err; exit 1; }
echo "gloo4 ok"; cut -c1-200 $O/r04_selflaunch_gloo4.json
timeout -k 10 400 python -u bench.py --gpus 4 --dist-backend gloo --steps 3 --warmup 1 --no-cpu --exchange 1 > $O/r04_selflaunch_gloo4_exchange.json 2> $O/r04_selflaunch_gloo4_exchange.err || { echo "gloo4 exchange failed"; tail -5 $O/r04_selflaunch_gloo4_exchange.err; exit 1; }
echo "gloo4 exchange ok"; cut -c1-200 $O/r04_selflaunch_gloo4_exchange.json
