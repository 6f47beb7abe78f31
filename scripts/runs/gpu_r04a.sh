#!/bin/bash
# Round-4 GPU call A: the free diagnosis and the first tests of the round's
# new paths (seed rings, device generator, multi-GPU setup from HBM).
#   gpurun --timeout 1200 -- bash scripts/gpu_r04a.sh TAG
TAG=${1:-r04a}
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
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
# hipMalloc / hipFree with no ordering of the library's own (round-2 code)
MAMG_POISON=1 MAMG_FREE_MODE=plain run poison_plain 300 $PYT tests/test_gpu.py
# null-stream ordered temporaries (round 4 default)
MAMG_POISON=1 run poison_default 300 $PYT tests/test_gpu.py
run rings 900 $PYT tests/test_gpu_rings.py
run devgen 300 $PYT tests/test_gpu_dist.py -k "device"
echo "== done"
