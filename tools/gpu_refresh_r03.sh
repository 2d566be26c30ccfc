# Round-3 refresh of the builder-measured rows: C5 K1, C3 over
# 200 steps, C4, unpartitioned input, the C5 rollups, the host feed.
set -e
mkdir -p gpurun_out
SKIP_TESTS=1 SKIP_BENCH=1 MATRIX="--config c5;--config c3 --steps 200;--config c4;--exchange 1" bash tools/gpu_session.sh
timeout -k 10 600 python tools/bench_rollup.py > gpurun_out/rollup_c5.log 2>&1
tail -1 gpurun_out/rollup_c5.log
timeout -k 10 300 python tools/bench_host_feed.py > gpurun_out/host_feed.log 2>&1
tail -3 gpurun_out/host_feed.log
