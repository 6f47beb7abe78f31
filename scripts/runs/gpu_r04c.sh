#!/bin/bash
# Round-4 GPU call C: hipFree by buffer size (sub-allocated small blocks vs a
# whole-allocation unmap), and the poisoned handle sequences for the
# product's null-stream ordered lifetimes and round 2's plain hipFree.
#   gpurun --timeout 1200 -- bash scripts/gpu_r04c.sh TAG
TAG=${1:-r04c}
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
for b in 4096 65536 1048576 16777216; do run free_race_$b 60 ./bench/free_race 100 $b; done
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
MAMG_POISON=1 MAMG_FREE_MODE=plain run poison_plain 420 $PYT tests/test_gpu.py
MAMG_POISON=1 run poison_default 420 $PYT tests/test_gpu.py
echo "== done"
