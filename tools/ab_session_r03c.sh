set -e
timeout -k 10 300 python -u -m pytest tests/test_k1_partitioned.py -k "pipelined" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
echo "== C3: host launches vs one many-batch call with pass C beside the next pass A on CU-partitioned streams"
ROUNDS=2 OPTS=" ;--persistent 1 --opt part_overlap=3;--persistent 1 --opt part_overlap=3 --opt part_ccus=32;--persistent 1 --opt part_overlap=3 --opt part_ccus=128;--persistent 1 --opt part_overlap=2" bash tools/ab_opts.sh
