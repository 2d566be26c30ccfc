#!/bin/bash
# multi-rank rehearsal of bench.py on a one-GPU box (gloo; the driver's node uses RCCL)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --no-cpu > gpurun_out/multi2.json 2> gpurun_out/multi2.err
rc=$?; echo "2 ranks rc=$rc"; cut -c1-400 gpurun_out/multi2.json; python -c "
import json; d=json.load(open('gpurun_out/multi2.json')); print('check', d.get('check')); print(d['config']['hll_keys_per_gpu'], d['value'])"
if [ $rc -ne 0 ]; then tail -30 gpurun_out/multi2.err; fi
exit $rc
