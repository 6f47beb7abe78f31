#!/bin/bash
# Round-4 GPU call E: name the array behind the poisoned handle failures
# (MAMG_DEBUG_SUMS prints each handle's operator hashes at upload and apply).
#   gpurun --timeout 900 -- bash scripts/gpu_r04e.sh TAG
TAG=${1:-r04e}
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
PYT="python -u -m pytest -v -s --timeout 200 --timeout-method thread"
K="k_kernel_variants"
MAMG_POISON=1 MAMG_DEBUG_SUMS=1 run sums_default 300 $PYT tests/test_gpu.py -k "$K"

MAMG_DEBUG_SUMS=1 run sums_nopoison 300 $PYT tests/test_gpu.py -k "$K"
echo "== done"
