#!/bin/bash
# C2 A/B: base library (tools/ab/libsketch_base.so) forked graph vs this tree forked graph vs persistent
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env, args
  timeout -k 10 120 env $2 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu --no-check $3 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$1 rc=$rc"; tail -5 gpurun_out/ab_$1.err; exit $rc; fi
  python -c "import json;d=json.load(open('gpurun_out/ab_$1.json'));r=d['roofline'];print('$1', round(d['value']/1e9,1), 'G/s ms/step', round(d['ms_per_step']*1e3,2), 'us dev', round(r['device_ms_per_step']*1e3,2), 'kern', round(r['kernel_ms']*1e3,2))"
}
for rep in 1 2; do
  run base$rep "SKE_LIB=tools/ab/libsketch_base.so" "--persistent 0"
  run fork$rep "X=1" "--persistent 0"
  run pers$rep "X=1" ""
  run pers_s$rep "X=1" "--steps 200 --max-batches 64"
done
