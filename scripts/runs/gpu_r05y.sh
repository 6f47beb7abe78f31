#!/bin/bash
# Round-5 GPU call Y: the reference family's GPU setup phases (its HEM
# aggregation went 0.9 -> 5.4 s in the r05z bench) with the round's SpGEMM
# staging / pairs switched off one at a time; then part 2 of the final
# check (trace, PMC, 8-rank rehearsal).
OUT=$(pwd)/gpurun_out/r05y
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  cat "$OUT/$name.log" | grep wall_s | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step s_def 300 python -u bench/ref_setup_phases.py 6 2
MAMG_SPGEMM_STAGE_GB=0 step s_nostage 300 python -u bench/ref_setup_phases.py 6 2
MAMG_SPGEMM_PAIR=0 step s_nopair 300 python -u bench/ref_setup_phases.py 6 2
echo "== done"
