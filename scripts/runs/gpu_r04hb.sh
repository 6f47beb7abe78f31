#!/bin/bash
# Round-4 A/B: sub-bands per XCD of the half-symmetric residual's band
# schedule (MAMG_HALF_BANDS 1 default, 2, 4) with the non-temporal read-once
# streams: alternating bench runs, one FETCH_SIZE pass each.
TAG=${1:-r04hb}
OUT=$(pwd)/gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
B="--steps 10 --warmup 2 --cpu-sample 0 --pcg 0 --compare-profiles 0"
step() {
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then echo "STOP ($rc)"; exit $rc; fi
}
for i in 1 2; do
  for v in 1 2 4; do
    MAMG_HALF_BANDS=$v step bench_b${v}_$i 300 python -u bench.py $B
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_b${v}_$i.log').read().strip().splitlines()[-1]); b=d['breakdown']; print('bands$v $i', d['value'], b['L0_resid']['ms'], b['L0_smooth_spmv']['ms'], b['L0_restrict']['ms'])" | tee -a $OUT/steps.log
  done
done
for v in 1 2 4; do
  cd /tmp && MAMG_HALF_BANDS=$v step pmc_b$v 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_b$v -o bench \
      -- python3 $ROOT/bench.py $B --no-breakdown; cd $ROOT
done
echo "== done"
