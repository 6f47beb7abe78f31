#!/bin/bash
# Round-5 GPU call X: the coarse tail launched with L2 affinity (8 workgroups,
# the first ticket runs it, the ones off XCD 0 wait ~7 us): tail / GS tests,
# then the reference family's W-cycle per apply with MAMG_TAIL_AFFINITY 1 / 0
# alternating (bench/prof_ref_family.py, nrefs=6, tail from 1024 nodes).
OUT=$(pwd)/gpurun_out/r05x
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step t_tail 600 python -u -m pytest tests/test_gpu_gs.py tests/test_gpu_configs.py tests/test_gpu_setup.py -x -q --timeout 200 --timeout-method thread
for k in a b; do
  MAMG_TAIL_AFFINITY=1 step a1$k 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 5
  MAMG_TAIL_AFFINITY=0 step a0$k 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 5
done
echo "== done"
# level 1 (623 K node rows) as multi-lane SELL (MAMG_MSELL_MIN_ROWS), the other coarse levels as before
B="python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 10"
for k in a b; do
  MAMG_MSELL_MIN_ROWS=500000 step m1$k 300 $B
  step m0$k 300 $B
done
echo "== done 2"
