#!/bin/bash
# Round-5 GPU call D: (1) the library's allocation log of the E16 handle
# sequence (diagnosis build, plain hipMalloc: no fault) and its replay with
# hipMalloc / contiguous re-homed streams / all contiguous (bench/alloc_replay);
# (2) the child-process tests on the diagnosis build; (3) patch setup timing.
TAG=${1:-r05d}
OUT=$(pwd)/gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
MAMG_LIB=$ROOT/metric-amg-examples_amd/libmamg_diag.so MAMG_ALLOC_LOG=$OUT/alloc.log \
  step alloclog 300 python -u -m pytest tests/test_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread -k test_k_kernel_variants
wc -l $OUT/alloc.log
step replay0 300 bench/alloc_replay $OUT/alloc.log 0
step replay1 300 bench/alloc_replay $OUT/alloc.log 1
step replay2 300 bench/alloc_replay $OUT/alloc.log 2
step children 900 python -u -m pytest tests/test_gpu_poison.py -q -x -p no:cacheprovider --timeout 900 --timeout-method thread
step patch 400 python -u bench/prof_patch_setup.py --nrefs 6
echo "== done"
