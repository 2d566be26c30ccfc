#!/bin/bash
# session-2 check: partitioned parity (pre-biased pass-A counters, tree-select
# pass B), many-batch and error-channel tests, then the default bench and the
# many-batch bench (branch streams no longer made for the partitioned K1)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_k1_partitioned.py tests/test_full_size.py tests/test_gpu_parity.py > gpurun_out/s2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/s2_tests.log; if [ $rc -ne 0 ]; then grep -B5 -A30 "^____" gpurun_out/s2_tests.log | head -60; exit $rc; fi
for mode in host many host many; do
  extra=""; [ $mode = many ] && extra="--persistent 1"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu $extra > gpurun_out/s2_$mode.json 2> gpurun_out/s2_$mode.err
  rc=$?; if [ $rc -ne 0 ]; then tail -5 gpurun_out/s2_$mode.err; exit $rc; fi
  python - gpurun_out/s2_$mode.json $mode <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["passes"]
print(sys.argv[2], "%.4e/s ms/step %.4f" % (d["value"], d["ms_per_step"]), " ".join("%s %.4f" % (k, v["ms"]) for k, v in p.items()), "check", d.get("check",{}).get("ok"), "rsb", d["roofline"].get("random_sector_bound",{}).get("frac"))
PY
done
