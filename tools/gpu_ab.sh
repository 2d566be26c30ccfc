#!/bin/bash
# One parameterised GPU session (replaces round 4-5's one-off
# tools/gpu_session_r0*.sh scripts): optional parity tests, then bench lines
# of several library builds alternated REPS times, for each argument set of
# MATRIX, then the per-pass table.  Every GPU step has its own time limit and
# the first failure ends the session.
#
#   TAG=r06a                      output prefix under gpurun_out/
#   TESTS="tests/a.py tests/b.py" pytest targets (-m gpu), "" to skip; "all": the whole GPU suite
#   SMOKE=1                       also __graft_entry__.smoke()
#   LIBS="new= base=tools/ab/libsketch_base.so"   name=SKE_LIB pairs ("" = in-tree build)
#   REPS=2                        alternations
#   MATRIX="--shard 8;"           ';'-separated extra bench argument sets ("" = the default step)
#   BENCH="--no-cpu --secondary none --host-fed 0"   common bench arguments
#   PROF=1                        rocprofv3 --kernel-trace --stats of the first LIBS entry, first MATRIX set
#   PMC="name=counters;..."       rocprofv3 --pmc passes of the first LIBS entry (one run per pass)
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
TAG=${TAG:-ab}
REPS=${REPS:-2}
BENCH=${BENCH:---no-cpu --secondary none --host-fed 0}
nproc > $O/${TAG}_host.txt
if [ -n "$TESTS" ]; then
  T=$TESTS; [ "$T" = all ] && T=tests
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -1 $O/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra SETS <<< "${MATRIX-}"
[ ${#SETS[@]} -eq 0 ] && SETS=("")
files=()
si=0
for v in "${SETS[@]}"; do
  for i in $(seq $REPS); do
    for nl in $LIBS; do
      name=${nl%%=*}; lib=${nl#*=}
      out=$O/${TAG}_m${si}_${name}_$i.json
      SKE_LIB=$lib timeout -k 10 300 python -u bench.py $BENCH $v > $out 2> ${out%.json}.err || { echo "bench [$name $v] failed"; tail -5 ${out%.json}.err; exit 1; }
      files+=($out)
    done
  done
  si=$((si + 1))
done
[ ${#files[@]} -gt 0 ] && python tools/r05_passes.py "${files[@]}"
first=${LIBS%% *}; flib=${first#*=}
if [ -n "$PROF" ]; then
  SKE_LIB=$flib timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_trace -o run --output-format csv -- python bench.py $BENCH ${SETS[0]} > $O/${TAG}_trace.log 2>&1 || { echo "trace failed"; tail -5 $O/${TAG}_trace.log; exit 1; }
  echo "trace ok"
fi
if [ -n "$PMC" ]; then
  IFS=';' read -ra PS <<< "$PMC"
  ARGS="--steps 4 --warmup 2 --no-cpu --no-check --secondary none --pass-replay 0 --host-fed 0 ${SETS[0]}"
  for p in "${PS[@]}"; do
    pn=${p%%=*}; ctrs=${p#*=}
    SKE_LIB=$flib timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $O/${TAG}_pmc_$pn -o run --output-format csv -- python bench.py $ARGS > $O/${TAG}_pmc_$pn.log 2>&1 || { echo "pmc $pn failed"; tail -3 $O/${TAG}_pmc_$pn.log; exit 1; }
    echo "pmc $pn ok"
  done
fi
exit 0
