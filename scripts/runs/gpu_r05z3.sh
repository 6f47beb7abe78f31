#!/bin/bash
# Round-5 GPU call Z3: the sampled pair check (setup tests, bench setup
# phases), then the 8-rank compute-only rehearsal (exchanges skipped) with
# level 0's K split around the coarse-e halo.
OUT=$(pwd)/gpurun_out/r05z3
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
step t_setup 400 python -u -m pytest tests/test_gpu_setup.py -x -q --timeout 200 --timeout-method thread
step b1 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown
step s_ref 300 python -u bench/ref_setup_phases.py 6 2
MAMG_DIST_TEST=dry step dry8 600 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --source device
echo "== done"
