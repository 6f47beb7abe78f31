#!/bin/bash
# K-kernel diagnosis: variants on one upload, then PMC
# passes below L2 (fabric read latency, DRAM share, TLB, TCP->TCC latency)
# over a light bench run.  From the repo root on an MI355X box:
#   gpurun --timeout 900 -- bash scripts/gpu_kdiag.sh TAG [STEPS]
# STEPS (default kvar,pmc): kvar = bench/kvariants.py; pmc = three --pmc passes.
TAG=${1:-kdiag}
STEPS=${2:-kvar,pmc}
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
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
LIGHT="--steps 10 --warmup 2 --cpu-sample 0 --no-breakdown --pcg 0 --compare-profiles 0"
want kvar && step kvar 400 python -u bench/kvariants.py --rounds 3 ${KVARS:-k0 k1 k2 k0r1}
if want pmc; then
  cd /tmp
  step pmc_ea 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_sum \
      TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum --output-format csv -d $OUT/pmc_ea -o bench -- python3 $ROOT/bench.py $LIGHT
  step pmc_tcp 150 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum \
      TCP_TCC_READ_REQ_sum --output-format csv -d $OUT/pmc_tcp -o bench -- python3 $ROOT/bench.py $LIGHT
  step pmc_sq 150 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES --output-format csv \
      -d $OUT/pmc_sq -o bench -- python3 $ROOT/bench.py $LIGHT
  cd $ROOT
  python3 scripts/pmc_summary.py $(find $OUT/pmc_ea $OUT/pmc_tcp $OUT/pmc_sq -name '*counter_collection.csv') \
      --json $OUT/pmc_summary.json > $OUT/pmc_summary.txt
  head -12 $OUT/pmc_summary.txt
fi
echo "== done"
