#!/bin/bash
# Round-4 GPU call E5-E9: the repeated level-0 AP conversion (MAMG_DEBUG_SUMS,
# values NaN-filled before the fill kernel) with three, two or one of the
# 48 KB csr2bsr workgroups per CU (MAMG_C2B_LDS_PAD).
#   gpurun --timeout 900 -- bash scripts/gpu_r04e5.sh TAG
TAG=${1:-r04e5}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
run() {   # run <name> <timeout> <cmd...>; stop on anything but pass/fail
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep -c 'blocks differ' $OUT/$name.txt) differing" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP ($rc)"; exit $rc; fi
}
PYT="python -u -m pytest -q -s --timeout 200 --timeout-method thread"
for i in 1 2 3; do
  MAMG_DEBUG_SUMS=1 run nopad_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
  MAMG_DEBUG_SUMS=1 MAMG_DEBUG_SYNC=1 run dsync_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
  MAMG_DEBUG_SUMS=1 MAMG_POISON=1 run poison_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
done
echo "== done"
