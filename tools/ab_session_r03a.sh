set -e
timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py -k "counter_layouts" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
ROUNDS=2 ARGS="--secondary none" LIBS="tools/ab/libsketch_base.so tools/ab/libsketch_abl8.so tools/ab/libsketch_abl16.so tools/ab/libsketch_abl24.so" bash tools/ab_passes.sh
ROUNDS=2 OPTS=" ;--opt pa_grid=3;--opt pa_grid=4;--opt pa_grid=5" bash tools/ab_opts.sh
echo "== C2 cold: base vs plain-store raises"
ROUNDS=2 ARGS="--config c2 --secondary none" LIBS="tools/ab/libsketch_base.so tools/ab/libsketch_k1st.so" bash tools/ab_passes.sh
echo "== C2 warm (100 warm-up steps)"
ROUNDS=1 ARGS="--config c2 --secondary none --warmup 100" LIBS="tools/ab/libsketch_base.so tools/ab/libsketch_k1st.so" bash tools/ab_passes.sh
echo "== casbench (XCD-local modes)"; timeout -k 10 120 ./tools/casbench | tee gpurun_out/casbench_r03.json
