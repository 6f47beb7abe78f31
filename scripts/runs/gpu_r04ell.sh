#!/bin/bash
# Round-4 A/B: the coarse tail's colour steps on ELL copies (tail_gs_ell,
# default) against the row-pointer path (MAMG_TAIL_ELL=0): the tail tests,
# then bench/prof_ref_family.py at nrefs=6 alternating.
TAG=${1:-r04ell}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(tail -1 $OUT/$name.log | cut -c1-200)" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then echo "STOP ($rc)"; exit $rc; fi
}
step tests 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gs.py tests/test_gpu_rings.py tests/test_gpu_configs.py
for i in 1 2; do
  MAMG_TAIL_ELL=0 step prof_ptr_$i 300 python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 1024 --op-profile
  step prof_ell_$i 300 python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 1024 --op-profile
done
echo "== done"
