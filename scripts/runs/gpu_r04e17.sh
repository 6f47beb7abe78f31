#!/bin/bash
# Round-4 GPU call E17: own temporary-block cache, contiguous allocations off:
# the repeated-conversion check, the whole GPU suite, one bench run.
TAG=${1:-r04e17}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep -c 'blocks differ' $OUT/$name.txt) differing, $(grep -c 'tmp_free' $OUT/$name.txt) tmp_free; $(tail -1 $OUT/$name.txt)" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then echo "STOP ($rc)"; exit $rc; fi
}
PYT="python -u -m pytest -q -s --timeout 200 --timeout-method thread"
for i in 1 2 3; do
  MAMG_DEBUG_SUMS=1 run kvar_$i 200 $PYT tests/test_gpu.py -k k_kernel_variants
done
run suite 900 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests
run bench 300 python -u bench.py
echo "== done"
