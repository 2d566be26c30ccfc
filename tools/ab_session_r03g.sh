set -e
timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
echo "== C3 pass C: fixed-count memory operations (in-tree) vs before (pc0)"
ROUNDS=3 ARGS="--secondary none" LIBS="tools/ab/libsketch_pc0.so real-time-student-attendance-system_amd/csrc/libsketch.so" bash tools/ab_passes.sh
