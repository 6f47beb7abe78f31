#!/bin/bash
# Round-4 A/B: lanes per row inside the coarse tail (MAMG_TAIL_VL 2 / 4
# (default) / 8) for the reference family's W-cycle, bench/prof_ref_family.py.
TAG=${1:-r04vl}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep -E '^ms/apply' $OUT/$name.log | tail -1)" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then echo "STOP ($rc)"; exit $rc; fi
}
for i in 1 2; do
  for v in 4 2 8; do
    MAMG_TAIL_VL=$v step prof_vl${v}_$i 300 python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 1024
  done
done
echo "== done"
