#!/bin/bash
# Round-5 GPU call F: smoke and the whole GPU suite on the current tree.
TAG=${1:-r05f}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step tests 1080 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
echo "== done"
