#!/bin/bash
# Round-4 GPU call E5: the repeated level-0 AP conversion (MAMG_DEBUG_SUMS)
# under the three free modes, twice each: which lifetimes give zeros.
#   gpurun --timeout 900 -- bash scripts/gpu_r04e5.sh TAG
TAG=${1:-r04e5}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
run() {   # run <name> <timeout> <cmd...>; stop on anything but pass/fail
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  grep -c "blocks differ" "$OUT/$name.txt" | sed 's/^/   conversions differing: /'
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP ($rc)"; exit $rc; fi
}
PYT="python -u -m pytest -q -s --timeout 200 --timeout-method thread"
for i in 1 2 3; do
  MAMG_DEBUG_SUMS=1 MAMG_FREE_MODE=drain run drain_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
  MAMG_DEBUG_SUMS=1 run default_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
  MAMG_DEBUG_SUMS=1 MAMG_FREE_MODE=plain run plain_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
done
echo "== done"
