#!/bin/bash
# Round-5 GPU call R: the pair-row staged SpGEMM count pass: bitwise tests,
# the GPU setup file, then setup timings with MAMG_SPGEMM_PAIR 1 / 0 alternating.
OUT=$(pwd)/gpurun_out/r05r
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
step t_setup 600 python -u -m pytest tests/test_gpu_setup.py tests/test_gpu_gs.py tests/test_gpu_blocks.py -x -q --timeout 200 --timeout-method thread
B="python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown"
for k in a b; do
  step p1$k 300 $B
  MAMG_SPGEMM_PAIR=0 step p0$k 300 $B
done
echo "== done"
