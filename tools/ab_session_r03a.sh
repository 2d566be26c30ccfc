set -e
timeout -k 10 600 python -u -m pytest tests/test_k1_partitioned.py tests/test_gpu_parity.py tests/test_processor.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
echo "== 2-rank gloo rehearsal (bench verify: owner-routed + SwipeExchange)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu --secondary none > gpurun_out/rehearsal2.log 2>&1
python -c "import json; d=json.loads(open('gpurun_out/rehearsal2.log').read().strip().splitlines()[-1]); c=d['check']; print('check ok', c['ok'], 'exchange ok', c['exchange']['ok'], c['exchange']['input'])"
ROUNDS=2 ARGS="--secondary none" LIBS="tools/ab/libsketch_base.so tools/ab/libsketch_abl8.so tools/ab/libsketch_abl16.so tools/ab/libsketch_abl24.so" bash tools/ab_passes.sh
ROUNDS=2 OPTS=" ;--opt pa_grid=3;--opt pa_grid=4;--opt pa_grid=5" bash tools/ab_opts.sh
echo "== C2 cold: base vs plain-store raises"
ROUNDS=2 ARGS="--config c2 --secondary none" LIBS="tools/ab/libsketch_base.so real-time-student-attendance-system_amd/csrc/libsketch.so tools/ab/libsketch_k1st.so" bash tools/ab_passes.sh
echo "== C2 warm (100 warm-up steps)"
ROUNDS=1 ARGS="--config c2 --secondary none --warmup 100" LIBS="tools/ab/libsketch_base.so real-time-student-attendance-system_amd/csrc/libsketch.so" bash tools/ab_passes.sh
echo "== casbench (XCD-local modes)"; timeout -k 10 120 ./tools/casbench | tee gpurun_out/casbench_r03.json
