set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/r06c_gpu_tests.log 2>&1; rc=$?
echo "gpu suite rc=$rc"; tail -2 $O/r06c_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r06c_smoke.log 2>&1 || { echo smoke failed; tail -5 $O/r06c_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py > $O/r06c_bench.json 2> $O/r06c_bench.err || { echo "bench failed"; tail -5 $O/r06c_bench.err; exit 1; }
python tools/r05_passes.py $O/r06c_bench.json
timeout -k 10 400 python -u bench.py --config c5 --no-cpu --secondary none --host-fed 0 > $O/r06c_c5.json 2> $O/r06c_c5.err || { echo "c5 failed"; tail -5 $O/r06c_c5.err; exit 1; }
echo c5 ok
timeout -k 10 400 python -u bench.py --gpus 8 --dist-backend gloo --steps 3 --warmup 1 --ownership mass --no-cpu --secondary none > $O/r06c_gloo8_mass.json 2> $O/r06c_gloo8_mass.err || { echo "gloo8 failed"; tail -5 $O/r06c_gloo8_mass.err; exit 1; }
echo gloo8 ok
timeout -k 10 500 python -u bench.py --config c5 --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu --secondary none --host-fed 0 > $O/r06c_c5_gloo2.json 2> $O/r06c_c5_gloo2.err || { echo "c5 gloo2 failed"; tail -5 $O/r06c_c5_gloo2.err; exit 1; }
echo c5gloo2 ok
