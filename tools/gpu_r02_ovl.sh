#!/bin/bash
# A/B of the pipelined many-batch partitioned K1 (C3, 20 steps in one call):
# serial, pass C beside the next B (part_overlap 1), beside the next A (2),
# and pass A at one block per CU beside C
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_k1_partitioned.py -k "many or pipelined" > gpurun_out/ovl_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ovl_tests.log; if [ $rc -ne 0 ]; then grep -B5 -A30 "^____" gpurun_out/ovl_tests.log | head -60; exit $rc; fi
run() {  # tag, args...
  tag=$1; shift
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu "$@" > gpurun_out/ovl_$tag.json 2> gpurun_out/ovl_$tag.err
  rc=$?; if [ $rc -ne 0 ]; then tail -5 gpurun_out/ovl_$tag.err; exit $rc; fi
  python - gpurun_out/ovl_$tag.json $tag <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["passes"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], " ".join("%s %.4f" % (k, v["ms"]) for k, v in p.items()), "check", d.get("check",{}).get("ok"))
PY
}
run host
run many0 --persistent 1
run ovl1 --persistent 1 --opt part_overlap=1
run ovl2 --persistent 1 --opt part_overlap=2
run ovl2g1 --persistent 1 --opt part_overlap=2 --opt pa_grid=1
run ovl2t0 --persistent 1 --opt part_overlap=2 --pass-timing 0
run ovl2g1t0 --persistent 1 --opt part_overlap=2 --opt pa_grid=1 --pass-timing 0
run host2
