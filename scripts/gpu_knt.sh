#!/bin/bash
# K-kernel non-temporal variants (device.hip launch_kvariant 4 / 5): timing
# round-robin on one upload, then FETCH_SIZE / WRITE_SIZE per variant.
#   gpurun --timeout 900 -- bash scripts/gpu_knt.sh TAG
TAG=${1:-knt}
OUT=$(pwd)/gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step <name> <timeout-seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step kvar 400 python -u bench/kvariants.py --rounds 3 ${KVARS:-k0 k4 k5}
cd /tmp
step pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o kv -- python3 $ROOT/bench/kvariants.py --rounds 1 --reps 3 ${KVARS:-k0 k4 k5}
step pmc_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o kv -- python3 $ROOT/bench/kvariants.py --rounds 1 --reps 3 ${KVARS:-k0 k4 k5}
cd $ROOT
echo "== done"
