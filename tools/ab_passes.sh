#!/bin/bash
# A/B of libsketch builds on one box with the partitioned K1's per-pass times:
# ROUNDS alternations of bench.py over LIBS, extra bench args in ARGS.
mkdir -p gpurun_out
LIBS=${LIBS:-"tools/ab/libsketch_base.so real-time-student-attendance-system_amd/csrc/libsketch.so"}
for r in $(seq ${ROUNDS:-3}); do
  for lib in $LIBS; do
    SKE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-check $ARGS > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
p = d["roofline"].get("passes", {})
print("%-48s %.4e/s  %.4f ms/step  %s" % (sys.argv[1].split("/")[-1], d["value"], d["ms_per_step"],
      " ".join("%s %.4f" % (k, v["ms"]) for k, v in p.items())))
PY
  done
done
