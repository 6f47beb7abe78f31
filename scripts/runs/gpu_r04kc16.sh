#!/bin/bash
# Round-4 A/B: level-0 K columns as 16-bit offsets from a per-slice base
# (MAMG_K_COL16=1, default) against int32 columns (MAMG_K_COL16=0): test_gpu.py,
# alternating bench runs, one FETCH_SIZE pass each.
TAG=${1:-r04kc16}
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
    MAMG_K_COL16=$v step bench_c${v}_$i 300 python -u bench.py $B
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_c${v}_$i.log').read().strip().splitlines()[-1]); b=d['breakdown']; print('c16_$v $i', d['value'], b['L0_resid']['ms'], b['L0_smooth_spmv']['ms'], b['L0_restrict']['ms'], d['k_region'])" | tee -a $OUT/steps.log
  done
done
for v in 0 1; do
  cd /tmp && MAMG_K_COL16=$v step pmc_c$v 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_c$v -o bench \
      -- python3 $ROOT/bench.py $B --no-breakdown; cd $ROOT
done
echo "== done"
