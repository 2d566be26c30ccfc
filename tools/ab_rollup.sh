#!/bin/bash
# A/B of libsketch builds on the C5 rollups (tools/bench_rollup.py), LIBS / ROUNDS / ARGS
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for lib in $LIBS; do
    SKE_LIB=$lib timeout -k 10 300 python tools/bench_rollup.py ${ARGS:---swipes 160000000} > gpurun_out/abr.json 2> gpurun_out/abr.err || { tail -5 gpurun_out/abr.err; exit 1; }
    python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abr.json").read().strip().splitlines()[-1])
print("%-24s" % sys.argv[1].split("/")[-1], " ".join("%s %.3f ms" % (k, v["kernel_s"] * 1e3) for k, v in d.items() if isinstance(v, dict) and "kernel_s" in v))
PY
  done
done
