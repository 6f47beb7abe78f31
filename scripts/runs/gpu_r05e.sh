#!/bin/bash
# Round-5 GPU call E: the distributed apply as a hipGraph (RCCL calls inside
# the capture): dist tests, 8-rank rehearsal (graph = eager bitwise at
# nrefs=6) and the dry per-rank compute time eager vs graph.
TAG=${1:-r05e}
OUT=$(pwd)/gpurun_out/$TAG
ROOT=$(pwd)
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
step dist_tests 900 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 300 --timeout-method thread
step rehearsal 600 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --source device
MAMG_DIST_TEST=dry step dry 600 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --source device
echo "== done"
