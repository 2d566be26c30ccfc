#!/bin/bash
# 4-rank rehearsal of the default bench (C3 shard per rank) on a one-GPU box (gloo)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29521 \
  bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo --no-cpu > gpurun_out/multi4.json 2> gpurun_out/multi4.err
rc=$?; echo "4 ranks rc=$rc"; grep '^{' gpurun_out/multi4.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['check'], d['config']['hll_keys_per_gpu'], {k: round(v['ms'],3) for k, v in d['roofline']['passes'].items()})"
if [ $rc -ne 0 ]; then tail -30 gpurun_out/multi4.err; fi
exit $rc
