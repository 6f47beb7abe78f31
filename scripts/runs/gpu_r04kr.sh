#!/bin/bash
# Round-4 A/B: K value region search (MAMG_KREGION_TRIES=4, default) against
# plain re-homing (1) with plain hipMalloc allocations: alternating bench runs.
TAG=${1:-r04kr}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
B="--steps 20 --warmup 3 --cpu-sample 0 --pcg 0 --compare-profiles 0"
step() {
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then echo "STOP ($rc)"; exit $rc; fi
}
for i in 1 2 3; do
  for v in 4 1; do
    MAMG_KREGION_TRIES=$v step bench_t${v}_$i 300 python -u bench.py $B
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_t${v}_$i.log').read().strip().splitlines()[-1]); b=d['breakdown']; print('tries$v $i', d['value'], b['L0_smooth_spmv']['ms'], d['setup']['wall_s'], d['setup']['phases_ms']['layout_kregion'], d['k_region'])" | tee -a $OUT/steps.log
  done
done
echo "== done"
