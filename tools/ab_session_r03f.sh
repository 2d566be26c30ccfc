set -e
timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py tests/test_full_size.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
echo "== C3 pass B boundary-load forms (v1 new pass A only, v2 + branch-free boundary offsets, v3 + ping-pong buffers, in-tree + unrolled group)"
ROUNDS=3 ARGS="--secondary none" LIBS="tools/ab/libsketch_v1.so tools/ab/libsketch_v2.so tools/ab/libsketch_v3.so real-time-student-attendance-system_amd/csrc/libsketch.so" bash tools/ab_passes.sh
