#!/bin/bash
# Round-4 A/B: the coarse tail for the Jacobi family from the last levels
# only (MAMG_TAIL_NODES=100 / 1000: levels 3-4 / 3-4 of nrefs=6) against no
# tail (default): alternating bench runs.
TAG=${1:-r04tj}
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
for i in 1 2; do
  step bench_none_$i 300 python -u bench.py $B
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_none_$i.log').read().strip().splitlines()[-1]); b=d['breakdown']; print('none $i', d['value'], d['graph_ms_per_step'], b['coarse_levels']['ms'])" | tee -a $OUT/steps.log
  for v in 100 8000; do
    MAMG_TAIL_NODES=$v step bench_t${v}_$i 300 python -u bench.py $B
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_t${v}_$i.log').read().strip().splitlines()[-1]); b=d['breakdown']; print('tail$v $i', d['value'], d['graph_ms_per_step'], b['coarse_levels']['ms'])" | tee -a $OUT/steps.log
  done
done
echo "== done"
