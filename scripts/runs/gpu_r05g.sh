#!/bin/bash
# Round-5 GPU call G: the N=1 bench (default flags, staged A0 upload), its
# kernel trace, the drivers' -precond metric sizes, the patch setup.
TAG=${1:-r05g}
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
step bench 600 python -u bench.py
tail -1 $OUT/bench.log > $OUT/bench.json
LIGHT="--steps 10 --warmup 2 --cpu-sample 0 --no-breakdown --pcg 0 --compare-profiles 0"
cd /tmp && step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench \
    -- python3 $ROOT/bench.py $LIGHT; cd $ROOT
step metric_sizes 400 python -u bench/precond_metric_sizes.py --max-n 128
step patch 300 python -u bench/prof_patch_setup.py --nrefs 6 --applies 3
echo "== done"
