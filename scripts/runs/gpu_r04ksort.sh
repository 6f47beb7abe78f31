#!/bin/bash
# Round-4 A/B: level-0 K rows sorted by length inside each SELL slice
# (MAMG_K_SORT=1, default) against row order (MAMG_K_SORT=0): test_gpu.py,
# alternating bench runs, one FETCH_SIZE pass each.
TAG=${1:-r04ksort}
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
  echo "== $name rc=$rc $(tail -1 $OUT/$name.log | cut -c1-150)" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then echo "STOP ($rc)"; exit $rc; fi
}
step tests 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py
for i in 1 2; do
  for v in 0 1; do
    MAMG_K_SORT=$v step bench_s${v}_$i 300 python -u bench.py $B
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_s${v}_$i.log').read().strip().splitlines()[-1]); b=d['breakdown']; print('sort$v $i', d['value'], b['L0_resid']['ms'], b['L0_smooth_spmv']['ms'], b['L0_restrict']['ms'], d['k_region'])" | tee -a $OUT/steps.log
  done
done
for v in 0 1; do
  cd /tmp && MAMG_K_SORT=$v step pmc_s$v 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_s$v -o bench \
      -- python3 $ROOT/bench.py $B --no-breakdown; cd $ROOT
done
echo "== done"
