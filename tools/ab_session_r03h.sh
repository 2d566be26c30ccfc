set -e
timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
echo "== C3 fixed-width layout: pass A templated on the id form (in-tree) vs HEAD"
ROUNDS=2 ARGS="--secondary none --layout fixed" LIBS="tools/ab/libsketch_head.so real-time-student-attendance-system_amd/csrc/libsketch.so" bash tools/ab_passes.sh
echo "== C3 offsets layout"
ROUNDS=2 ARGS="--secondary none" LIBS="tools/ab/libsketch_head.so real-time-student-attendance-system_amd/csrc/libsketch.so" bash tools/ab_passes.sh
