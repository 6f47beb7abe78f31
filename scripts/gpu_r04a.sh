#!/bin/bash
# Round-4 GPU call A: the free diagnosis (scripts/gpu_freediag.sh steps) and
# the first seed-ring Schwarz GPU tests.
#   gpurun --timeout 1200 -- bash scripts/gpu_r04a.sh TAG
TAG=${1:-r04a}
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
run free_race 90 ./bench/free_race 200
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
MAMG_POISON=1 MAMG_DRAIN=0 MAMG_FREELOG=1 run nodrain1 300 $PYT tests/test_gpu.py
MAMG_POISON=1 MAMG_DRAIN=0 run nodrain2 300 $PYT tests/test_gpu.py
run rings 600 $PYT tests/test_gpu_rings.py
echo "== done"
