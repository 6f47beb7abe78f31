#!/bin/bash
# Round-4 A/B: level-0 K kernel variants with the rows sorted inside slices
# (MAMG_K_VARIANT 0: two lanes per row, chunks of 5 (default); 2: four lanes,
# chunks of 3; 3: XCD-contiguous row order): alternating bench runs.
TAG=${1:-r04kv}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
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
  for v in 0 2 3; do
    MAMG_K_VARIANT=$v step bench_v${v}_$i 300 python -u bench.py $B
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_v${v}_$i.log').read().strip().splitlines()[-1]); b=d['breakdown']; print('kvar$v $i', d['value'], b['L0_resid']['ms'], b['L0_smooth_spmv']['ms'], d['k_region'])" | tee -a $OUT/steps.log
  done
done
echo "== done"
