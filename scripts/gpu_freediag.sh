#!/bin/bash
# Round-4 diagnosis of the round-3 intermittent wrong operators (VERDICT r03
# next-round #1): does hipFree wait for queued readers (bench/free_race), and
# does the poisoned test_gpu.py fail without the drain before each free
# (MAMG_DRAIN=0), with every free issued under pending work logged?
#   gpurun --timeout 600 -- bash scripts/gpu_freediag.sh TAG
TAG=${1:-fd}
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
PYT="python -u -m pytest tests/test_gpu.py -v --timeout 120 --timeout-method thread"
MAMG_POISON=1 MAMG_DRAIN=0 MAMG_FREELOG=1 run nodrain1 300 $PYT
MAMG_POISON=1 MAMG_DRAIN=0 run nodrain2 300 $PYT
MAMG_POISON=1 MAMG_DRAIN=1 MAMG_FREELOG=1 run drain 300 $PYT
echo "== done"
