#!/bin/bash
# Round-5 GPU call L: where the 8-rank reference-preset rehearsal crashed
# (host SIGSEGV after the setups, call K): nrefs=5 and 4 first, with the
# Python fault handler; each step stops the call on a crash.
OUT=$(pwd)/gpurun_out/r05l
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step s6_8 900 python -X faulthandler -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --profile schwarz
MAMG_DIST_TEST=dry step s6_8_dry 900 python -X faulthandler -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --profile schwarz
echo "== done"
