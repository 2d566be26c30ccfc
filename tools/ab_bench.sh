#!/bin/bash
# A/B of libsketch builds on one box: ROUNDS alternations of bench.py over the
# builds named in LIBS (default: tools/ab/libsketch_base.so and the in-tree
# build), extra bench args in ARGS.  Prints swipes/s and kernel us per line.
mkdir -p gpurun_out
LIBS=${LIBS:-"tools/ab/libsketch_base.so real-time-student-attendance-system_amd/csrc/libsketch.so"}
for r in $(seq ${ROUNDS:-3}); do
  for lib in $LIBS; do
    SKE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu $ARGS > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
print("%-60s %.4e swipes/s  kernel %.2f us" % (sys.argv[1], d["value"], d["roofline"]["kernel_ms"] * 1e3))
PY
  done
done
