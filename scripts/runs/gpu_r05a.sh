#!/bin/bash
# Round-5 GPU call A: smoke, the N=1 bench, and a kernel trace of the
# reference preset's node-patch setup.
TAG=${1:-r05a}
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
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py --cpu-sample 3 --compare-profiles 0
tail -1 $OUT/bench.log > $OUT/bench.json
step patch 400 python -u bench/prof_patch_setup.py --nrefs 6
cd /tmp && step patch_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/patch_trace -o p \
    -- python3 $ROOT/bench/prof_patch_setup.py --nrefs 6; cd $ROOT
echo "== done"
