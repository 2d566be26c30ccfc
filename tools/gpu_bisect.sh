#!/bin/bash
O=gpurun_out
timeout -k 10 120 python -u tools/diag_part.py 700333 > $O/diag_tree.log 2>&1; echo "diag rc=$?"; cat $O/diag_tree.log | grep -v amdgpu.ids
for v in al16 a4big; do
SKE_LIB=tools/ab/libsketch_$v.so timeout -k 10 200 python -u -m pytest tests/test_k1_partitioned.py -q --timeout 120 --timeout-method thread > $O/bis_$v.log 2>&1; echo "$v rc=$?"; tail -4 $O/bis_$v.log
done
