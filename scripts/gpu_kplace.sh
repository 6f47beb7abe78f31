#!/bin/bash
# K placement diagnosis: K timed after moving its value
# array between plain and physically contiguous allocations in one process,
# then the same moves under two rocprofv3 --pmc passes (fabric read latency /
# DRAM, TLB / TCP->TCC latency), summarised per placement.
#   gpurun --timeout 1200 -- bash scripts/gpu_kplace.sh TAG
TAG=${1:-kplace}
OUT=$(pwd)/gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step time 500 python -u bench/kplace.py --variants ${KVARS:-0} --moves ${MOVES:-val:2,val+:2,val:2,val+:2,col+:1,col:1}
PM="--reps 5 --moves val:1,val+:1,val:1,val+:1"
cd /tmp
step pmc_ea 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_sum \
    TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum --output-format csv -d $OUT/pmc_ea -o kp -- python3 $ROOT/bench/kplace.py $PM
step pmc_tcc 300 rocprofv3 --pmc TCC_TAG_STALL_sum TCC_LATENCY_FIFO_FULL_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_128B_sum \
    --output-format csv -d $OUT/pmc_tcc -o kp -- python3 $ROOT/bench/kplace.py $PM
step pmc_tcp 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum \
    TCP_TCC_READ_REQ_sum --output-format csv -d $OUT/pmc_tcp -o kp -- python3 $ROOT/bench/kplace.py $PM
cd $ROOT
python3 scripts/pmc_dispatch.py $(find $OUT/pmc_ea $OUT/pmc_tcc $OUT/pmc_tcp -name '*counter_collection.csv') \
    --kernel msell_kernel --groups 16,9,9,9,9 > $OUT/pmc_dispatch.txt
cat $OUT/pmc_dispatch.txt
echo "== done"
