#!/bin/bash
# Round-4 GPU call E13: the repeated AP conversion with the re-homed K
# regions in plain hipMalloc memory (MAMG_CONTIG=0) against physically
# contiguous allocations (default), interleaved.
TAG=${1:-r04e13}
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
  MAMG_DEBUG_SUMS=1 MAMG_CONTIG=0 run nocontig_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
  MAMG_DEBUG_SUMS=1 run contig_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
done
echo "== done"
