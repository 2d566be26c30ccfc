#!/bin/bash
# C2 persistent K1: steps / warmup sweep (register state vs per-step time)
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, args
  timeout -k 10 120 python bench.py --config c2 --no-cpu --no-check $2 > gpurun_out/sw_$1.json 2> gpurun_out/sw_$1.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$1 rc=$rc"; tail -5 gpurun_out/sw_$1.err; exit $rc; fi
  python -c "import json;d=json.load(open('gpurun_out/sw_$1.json'));r=d['roofline'];print('$1', round(d['value']/1e9,1), 'G/s ms/step', round(d['ms_per_step']*1e3,2), 'us dev', round(r['device_ms_per_step']*1e3,2), 'kern', round(r['kernel_ms']*1e3,2), r['passes']['k1']['launches'])"
}
run s20w5 "--steps 20 --warmup 5"
run s20w5b "--steps 20 --warmup 5"
run s48w5 "--steps 48 --warmup 5"
run s20w100 "--steps 20 --warmup 100 --max-batches 64"
run s20w5m64 "--steps 20 --warmup 5 --max-batches 64"
run s20w5g "--steps 20 --warmup 5 --persistent 0"
run s200w5g "--steps 200 --warmup 5 --persistent 0 --max-batches 64"
