#!/bin/bash
# Round-5 GPU call O: the one-pass (staged) hash SpGEMM of the GPU setup:
# its bitwise tests, the GPU setup file, then bench setup timings with
# staging on / off alternating (setup phases in the bench line).
OUT=$(pwd)/gpurun_out/r05o
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step t_stage 300 python -u -m pytest tests/test_gpu_setup.py -x -v --timeout 120 --timeout-method thread -k "staging"
step t_setup 600 python -u -m pytest tests/test_gpu_setup.py -x -q --timeout 200 --timeout-method thread
B="python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown"
for k in a b; do
  step s1$k 300 $B
  MAMG_SPGEMM_STAGE_GB=0 step s0$k 300 $B
done
echo "== done"
