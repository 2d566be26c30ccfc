mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu --streams 4 > gpurun_out/b4.log 2>&1 && tail -1 gpurun_out/b4.log | cut -c1-200 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python bench.py --no-cpu --streams 4 > gpurun_out/prof4.log 2>&1 && head -3 gpurun_out/prof4/run_kernel_stats.csv
