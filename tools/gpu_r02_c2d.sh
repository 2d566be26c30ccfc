#!/bin/bash
# C2 persistent K1 A/B: one-deep settle (tools/ab/libsketch_p1.so) vs this tree
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env, args
  timeout -k 10 120 env $2 python bench.py --config c2 --no-cpu --no-check $3 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$1 rc=$rc"; tail -5 gpurun_out/ab_$1.err; exit $rc; fi
  python -c "import json;d=json.load(open('gpurun_out/ab_$1.json'));r=d['roofline'];print('$1', round(d['value']/1e9,1), 'G/s ms/step', round(d['ms_per_step']*1e3,2), 'us dev', round(r['device_ms_per_step']*1e3,2), 'kern', round(r['kernel_ms']*1e3,2))"
}
for rep in 1 2; do
  run p1_$rep "SKE_LIB=tools/ab/libsketch_p1.so" "--steps 20 --warmup 5"
  run p2_$rep "X=1" "--steps 20 --warmup 5"
  run p1w_$rep "SKE_LIB=tools/ab/libsketch_p1.so" "--steps 20 --warmup 100 --max-batches 64"
  run p2w_$rep "X=1" "--steps 20 --warmup 100 --max-batches 64"
done
