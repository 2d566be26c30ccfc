#!/bin/bash
# 2048-swipe tiles for one-link k=11 chains: partitioned parity tests, then A/B against 1024-swipe tiles
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_k1_partitioned.py \
  "tests/test_full_size.py::test_c3_bench_shard_one_gpu" "tests/test_full_size.py::test_c3_gpu_shard_full_step" \
  "tests/test_full_size.py::test_c3_many_batches_graph" "tests/test_gpu_parity.py::test_swipes_c3_filter_vs_oracle" \
  "tests/test_gpu_parity.py::test_swipes_fixed_width_equals_offsets" > gpurun_out/t_tile.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_tile.log; if [ $rc -ne 0 ]; then tail -40 gpurun_out/t_tile.log; exit $rc; fi
for rep in 1 2; do
for v in 10 11; do
  timeout -k 10 200 python bench.py --no-cpu --no-check --pa-tile $v > gpurun_out/tile_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/tile_$v.json'));r=d['roofline'];print('tile=$v', round(d['ms_per_step'],4), {k:round(v['ms'],4) for k,v in r['passes'].items()})"
done; done
