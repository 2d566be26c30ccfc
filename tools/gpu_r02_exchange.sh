#!/bin/bash
# unpartitioned input (alltoallv routing): device parity test, 1-rank and 2-rank (gloo) bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_exchange_gpu.py > gpurun_out/t_ex.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_ex.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/t_ex.log; exit $rc; fi
timeout -k 10 300 python bench.py --exchange 1 --steps 5 --warmup 2 --no-cpu > gpurun_out/ex1.json 2> gpurun_out/ex1.err
rc=$?; echo "1 rank rc=$rc"; grep '^{' gpurun_out/ex1.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['check']['ok'], d['config']['input'], {k: round(v['ms'],3) for k, v in d['roofline']['passes'].items()})"
if [ $rc -ne 0 ]; then tail -20 gpurun_out/ex1.err; exit $rc; fi
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 \
  bench.py --gpus 2 --exchange 1 --steps 4 --warmup 1 --dist-backend gloo --no-cpu > gpurun_out/ex2.json 2> gpurun_out/ex2.err
rc=$?; echo "2 ranks rc=$rc"; grep '^{' gpurun_out/ex2.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['check'], d['config']['hll_keys_per_gpu'])"
if [ $rc -ne 0 ]; then tail -30 gpurun_out/ex2.err; fi
exit $rc
