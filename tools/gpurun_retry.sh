#!/bin/bash
# run one gpurun command, retrying ONLY when no box/slot was free (rc 3 or a
# "transient" status: nothing ran, nothing charged), at most 8 times
out=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  timeout 1500 /usr/local/graft/bin/gpurun --timeout 900 -- "$@" > "$out" 2>&1; rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then sleep 150; continue; fi
  exit $rc
done
exit 3
