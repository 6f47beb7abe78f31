#!/bin/bash
# Round-4 GPU call D: the coarse tail rework (512 threads, staged matrix
# slices, L2 warm-up): parity, then the reference family's W-cycle A/B.
#   gpurun --timeout 1200 -- bash scripts/gpu_r04d.sh TAG
TAG=${1:-r04d}
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
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
run tail_tests 500 $PYT tests/test_gpu.py tests/test_gpu_gs.py tests/test_gpu_configs.py -k "tail or w_cycle or gs or sgs"
R="python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 1024 --op-profile"
run ref_new 240 $R
MAMG_TAIL_NOSTAGE=1 run ref_nostage 240 $R
MAMG_TAIL_NOTOUCH=1 run ref_notouch 240 $R
MAMG_LIB=$(pwd)/ab/libmamg_r04base.so run ref_base 240 $R
run ref_t4096 240 python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 4096 --op-profile
echo "== done"
