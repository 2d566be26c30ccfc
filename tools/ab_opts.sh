#!/bin/bash
# A/B of library options on one box with the partitioned K1's per-pass times:
# ROUNDS alternations of bench.py over the ';'-separated option sets in OPTS
# (each a list of bench.py arguments, e.g. "--opt k1_grid=128"; an empty set is
# the default), extra bench args in ARGS, the library in SKE_LIB (default in-tree).
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${OPTS:-}"
for r in $(seq ${ROUNDS:-3}); do
  for v in "${SETS[@]}"; do
    timeout -k 10 200 python bench.py --no-cpu --no-check --secondary none $ARGS $v > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
p = d["roofline"].get("passes", {})
print("%-32s %.4e/s  %.4f ms/step  %s" % ("[" + sys.argv[1].strip() + "]", d["value"], d["ms_per_step"],
      " ".join("%s %.4f" % (k, v["ms"]) for k, v in p.items())))
PY
  done
done
