#!/bin/bash
# Round-4 A/B: hsell2_kernel's read-once streams as non-temporal loads
# (ab/libmamg_nt.so, -DMAMG_HSELL_NT=1) against the same tree without
# (ab/libmamg_base.so): alternating bench runs, then one FETCH_SIZE pass each.
TAG=${1:-r04nt}
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
  for v in base nt1 nt2; do
    MAMG_LIB=$ROOT/ab/libmamg_$v.so step bench_${v}_$i 300 python -u bench.py $B
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_${v}_$i.log').read().strip().splitlines()[-1]); b=d['breakdown']; print('$v $i', d['value'], b['L0_resid']['ms'], b['L0_smooth_spmv']['ms'], b['L0_restrict']['ms'])" | tee -a $OUT/steps.log
  done
done
for v in base nt1 nt2; do
  cd /tmp && MAMG_LIB=$ROOT/ab/libmamg_$v.so step pmc_$v 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$v -o bench \
      -- python3 $ROOT/bench.py $B --no-breakdown; cd $ROOT
done
echo "== done"
