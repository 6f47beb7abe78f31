#!/bin/bash
# Round-4 GPU call E12: the repeated AP conversion with every XCD's L2
# written back and invalidated (system-scope fence in 2048 workgroups)
# after the NaN fill (1) or after the conversion (2).
TAG=${1:-r04e12}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep -c 'blocks differ' $OUT/$name.txt) differing" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP ($rc)"; exit $rc; fi
}
PYT="python -u -m pytest -q -s --timeout 200 --timeout-method thread"
for i in 1 2 3; do
  MAMG_DEBUG_SUMS=1 MAMG_DEBUG_FLUSH=1 run flush_after_fill_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
  MAMG_DEBUG_SUMS=1 MAMG_DEBUG_FLUSH=2 run flush_after_conv_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
  MAMG_DEBUG_SUMS=1 run noflush_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
done
echo "== done"
