#!/bin/bash
# Round-5 GPU call B: node-patch colouring (incremental Jones-Plassmann) and
# readlane Gauss-Jordan: patch tests, setup time and kernel trace at nrefs=6.
TAG=${1:-r05c}
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
step patch_tests 600 python -u -m pytest tests/test_gpu_patch.py tests/test_gpu_rings.py -m gpu -x -q --timeout 200 --timeout-method thread
step patch 400 python -u bench/prof_patch_setup.py --nrefs 6 --applies 3
cd /tmp && step patch_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/patch_trace -o p \
    -- python3 $ROOT/bench/prof_patch_setup.py --nrefs 6; cd $ROOT
echo "== done"
