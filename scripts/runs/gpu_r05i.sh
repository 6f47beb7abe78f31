#!/bin/bash
# Round-5 GPU call I: A_0 upload A/B (staged vs the runtime's pageable copy),
# fresh processes alternating, diagnosis build.
OUT=$(pwd)/gpurun_out/r05i
mkdir -p $OUT
export MAMG_LIB=$(pwd)/metric-amg-examples_amd/libmamg_diag.so
for i in 1 2 3; do
  timeout -k 10 120 python -u bench/upload_ab.py 6 >> $OUT/ab.txt 2>&1 || exit $?
  MAMG_UPLOAD_PLAIN=1 timeout -k 10 120 python -u bench/upload_ab.py 6 >> $OUT/ab.txt 2>&1 || exit $?
done
grep wall_s $OUT/ab.txt
