#!/bin/bash
# persistent LDS K1 with deferred register CASes: C2 parity, then A/B cold and warm
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_full_size.py -k "c2 or c4" tests/test_gpu_parity.py > gpurun_out/t_c2e.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_c2e.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/t_c2e.log; exit $rc; fi
run() {  # name, env, args
  timeout -k 10 120 env $2 python bench.py --config c2 --no-cpu --no-check $3 > gpurun_out/c2e_$1.json 2> gpurun_out/c2e_$1.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$1 rc=$rc"; tail -5 gpurun_out/c2e_$1.err; exit $rc; fi
  python -c "import json;d=json.load(open('gpurun_out/c2e_$1.json'));r=d['roofline'];print('$1', round(d['value']/1e9,1), 'G/s ms/step', round(d['ms_per_step']*1e3,2), 'us kern/step', round(r['kernel_ms']*1e3/20,2))"
}
for rep in 1 2; do
  run base_cold$rep "SKE_LIB=tools/ab/libsketch_base.so" "--steps 20 --warmup 5"
  run new_cold$rep "X=1" "--steps 20 --warmup 5"
  run base_warm$rep "SKE_LIB=tools/ab/libsketch_base.so" "--steps 20 --warmup 100 --max-batches 64"
  run new_warm$rep "X=1" "--steps 20 --warmup 100 --max-batches 64"
done
