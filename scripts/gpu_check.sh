#!/bin/bash
# The GPU recipe: run on an MI355X box from the repo root,
#   gpurun --timeout 1200 -- bash scripts/gpu_check.sh TAG [STEPS]
# STEPS (default all): any of smoke tests bench trace pmc dist, comma-separated.
#   smoke  __graft_entry__.smoke()
#   tests  pytest -m gpu
#   bench  python bench.py (N = 1 defaults) -> gpurun_out/TAG/bench.json
#   trace  rocprofv3 --kernel-trace --stats of a bench run -> TAG/trace/*_kernel_stats.csv
#   pmc    rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE (separate passes) ->
#          scripts/traffic.py -> profiles/traffic.json (tagged with device.hip's sha256)
#   dist   bench/dist_rehearsal.py: 8 virtual ranks of nrefs=6, A0 generated in HBM
# Stops at the first crash / timeout / abort; logs in gpurun_out/TAG/.  Copy
# the summaries to be kept into profiles/ afterwards.
TAG=${1:-check}
STEPS=${2:-smoke,tests,bench,trace,pmc,dist}
OUT=$(pwd)/gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
want() { [[ ",$STEPS," == *",$1,"* ]]; }
step() {   # step <name> <timeout-seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
LIGHT="--steps 10 --warmup 2 --cpu-sample 0 --no-breakdown --pcg 0 --compare-profiles 0"
want smoke && step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
want tests && step tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
if want bench; then
  step bench 600 python -u bench.py && tail -1 $OUT/bench.log > $OUT/bench.json
fi
if want trace; then
  cd /tmp && step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench \
      -- python3 $ROOT/bench.py $LIGHT; cd $ROOT
fi
if want pmc; then
  cd /tmp && step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o bench \
      -- python3 $ROOT/bench.py $LIGHT; cd $ROOT
  cd /tmp && step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o bench \
      -- python3 $ROOT/bench.py $LIGHT; cd $ROOT
  F=$(find $OUT/pmc_fetch -name '*counter_collection.csv' | head -1)
  W=$(find $OUT/pmc_write -name '*counter_collection.csv' | head -1)
  BJ=""; [ -s $OUT/bench.json ] && BJ="--bench-json $OUT/bench.json"
  python3 scripts/traffic.py "$F" "$W" --N 33949186 $BJ --out $OUT/traffic.json && cp $OUT/traffic.json profiles/traffic.json
fi
want dist && step dist 600 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --source device
echo "== done"
