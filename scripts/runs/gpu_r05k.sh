#!/bin/bash
# Round-5 GPU call K: the reference preset (node patches on level 0) on 8
# virtual ranks of nrefs=6: result vs one GPU, per-rank compute (dry).
OUT=$(pwd)/gpurun_out/r05k
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step schwarz8 900 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --profile schwarz
MAMG_DIST_TEST=dry step schwarz8_dry 900 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --profile schwarz
echo "== done"
