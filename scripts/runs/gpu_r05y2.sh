#!/bin/bash
# Round-5 GPU call Y2: pairs only when most node row pairs agree (UA's R = T^T
# never does); the reference family's setup in a fresh process, then the
# bench's profile comparison (where the first HEM setup of the process took
# 5.4 s of aggregation) with and without SpGEMM staging.
OUT=$(pwd)/gpurun_out/r05y2
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  grep wall_s "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step t_setup 300 python -u -m pytest tests/test_gpu_setup.py -x -q --timeout 200 --timeout-method thread
step s_def 300 python -u bench/ref_setup_phases.py 6 2
step b_def 600 python -u bench.py --cpu-sample 0 --steps 5 --pcg 1 --compare-profiles 1
MAMG_SPGEMM_STAGE_GB=0 step b_nostage 600 python -u bench.py --cpu-sample 0 --steps 5 --pcg 1 --compare-profiles 1
echo "== done"
