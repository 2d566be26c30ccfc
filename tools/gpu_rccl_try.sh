#!/bin/bash
# experiment: RCCL with 2 ranks on one GPU (sharded queries, exchange)
set -o pipefail
O=gpurun_out
mkdir -p $O/rccl
WORKER_BACKEND=nccl NCCL_DEBUG=WARN timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29651 tests/sharded_worker.py $O/rccl/sharded.npz > $O/rccl/sharded.log 2>&1; echo "sharded nccl rc=$?"; tail -15 $O/rccl/sharded.log
