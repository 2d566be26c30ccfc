#!/bin/bash
# A/B: register pre-check in pass A (pa_precheck 1) against pass C's own loads (0),
# after the partitioned-K1 parity tests
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_k1_partitioned.py tests/test_full_size.py > gpurun_out/pre_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pre_tests.log; if [ $rc -ne 0 ]; then grep -B5 -A30 "^____" gpurun_out/pre_tests.log | head -80; exit $rc; fi
for pre in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --pa-precheck $pre > gpurun_out/pre_$pre.json 2> gpurun_out/pre_$pre.err
  rc=$?; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pre_$pre.err; exit $rc; fi
  python - gpurun_out/pre_$pre.json $pre <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["passes"]
print("pre", sys.argv[2], "ms/step %.4f" % d["ms_per_step"], " ".join("%s %.4f" % (k, v["ms"]) for k, v in p.items()), "check", d.get("check",{}).get("ok"))
PY
done
