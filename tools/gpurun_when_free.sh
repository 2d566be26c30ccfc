#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports no free
# slot / box (a transient refusal: nothing ran, nothing charged), at most
# $TRIES times, $WAIT s apart.  Any run that started is never repeated.
#   usage: bash tools/gpurun_when_free.sh <log> <timeout> '<command>'
log=$1; to=$2; cmd=$3
for i in $(seq ${TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  if grep -q "status=transient" $log && ! grep -q "run [1-9]" $log; then
    echo "[when_free] attempt $i: transient, waiting" >> $log.tries; sleep ${WAIT:-150}; continue
  fi
  break
done
echo done >> $log
