#!/bin/bash
# Round-4 A/B: launched GS colour steps with the row's own operands loaded
# before the block loop (gs2_kernel) against the previous order
# (ab/libmamg_base.so): GS / rings / config tests, then
# bench/prof_ref_family.py at nrefs=6 alternating.
TAG=${1:-r04gs}
OUT=$(pwd)/gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep -E '^ms/apply|passed|failed' $OUT/$name.log | tail -1 | cut -c1-120)" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then echo "STOP ($rc)"; exit $rc; fi
}
step tests 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gs.py tests/test_gpu_rings.py tests/test_gpu_configs.py tests/test_gpu_patch.py
for i in 1 2; do
  MAMG_LIB=$ROOT/ab/libmamg_base.so step prof_base_$i 300 python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 1024
  step prof_new_$i 300 python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 1024
done
echo "== done"
