#!/bin/bash
# A/B of library builds on one box with the partitioned K1's per-pass times:
# ROUNDS alternations of bench.py over the ';'-separated builds in LIBS
# (each name=path of a libsketch.so, e.g. base=tools/ab/libsketch_r03.so;
# "tree" = the in-tree build), extra bench args in ARGS.
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${LIBS:-tree=}"
for r in $(seq ${ROUNDS:-3}); do
  for v in "${SETS[@]}"; do
    name=${v%%=*}; lib=${v#*=}
    if [ -n "$lib" ]; then export SKE_LIB=$lib; else unset SKE_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu --no-check --secondary none $ARGS > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
p = d["roofline"].get("passes", {})
print("%-12s %.4e/s  %.4f ms/step  %s" % (sys.argv[1], d["value"], d["ms_per_step"],
      " ".join("%s %.4f" % (k, v["ms"]) for k, v in p.items())), flush=True)
PY
  done
done
