#!/bin/bash
# Round-4 GPU call F: coarse tail with the program in LDS: parity and the
# reference family's W-cycle against the round-3 tail (ab/libmamg_r04base.so).
#   gpurun --timeout 900 -- bash scripts/gpu_r04f.sh TAG
TAG=${1:-r04f}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
run() {   # run <name> <timeout> <cmd...>; stop on anything but pass/fail
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP ($rc)"; exit $rc; fi
}
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
run tail_tests 500 $PYT tests/test_gpu_gs.py -k "tail"
R="python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 1024 --op-profile"
run ref_new 240 $R
MAMG_LIB=$(pwd)/ab/libmamg_r04base.so run ref_base 240 $R
run ref_new2 240 $R
echo "== done"
