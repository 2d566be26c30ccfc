#!/bin/bash
# partitioned K1 A/B on C3: base library (tools/ab/libsketch_base.so) vs this tree, per-pass times
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_k1_partitioned.py "tests/test_full_size.py::test_c3_bench_shard_one_gpu" "tests/test_full_size.py::test_c3_many_batches_graph" "tests/test_full_size.py::test_c4_adversarial_step" > gpurun_out/t_ab3.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_ab3.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/t_ab3.log; exit $rc; fi
run() {  # name, env
  timeout -k 10 200 env $2 python bench.py --no-cpu --no-check $3 > gpurun_out/ab3_$1.json 2> gpurun_out/ab3_$1.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$1 rc=$rc"; tail -5 gpurun_out/ab3_$1.err; exit $rc; fi
  python -c "import json;d=json.load(open('gpurun_out/ab3_$1.json'));r=d['roofline'];print('$1', round(d['value']/1e9,2), 'G/s ms/step', round(d['ms_per_step'],4), {k:round(v['ms'],4) for k,v in r['passes'].items()})"
}
for rep in 1 2; do
  run base$rep "SKE_LIB=tools/ab/libsketch_base.so" ""
  run new$rep "X=1" ""
done
