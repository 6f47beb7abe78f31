#!/bin/bash
# Round-6 GPU call E: why level-0 K is slower inside the
# cycle than in the upload-time region chooser.  (a) kernel trace of a light
# bench (per-dispatch durations of the chooser's K launches and the timed
# cycle's); (b) one PMC pass (L2 hit / miss, fabric requests, UTCL1
# translations) of the same; (c) the light bench with PyTorch's caching
# allocator off (the caller's r / z from a plain hipMalloc each).
OUT=$(pwd)/gpurun_out/r06e
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
LIGHT="--steps 10 --warmup 2 --cpu-sample 0 --no-breakdown --pcg 0 --compare-profiles 0"
cd /tmp
step trace 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o bench -- python3 $ROOT/bench.py $LIGHT
step pmc 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv -d $OUT/pmc -o bench -- python3 $ROOT/bench.py $LIGHT
cd $ROOT
step light 300 python3 bench.py $LIGHT
PYTORCH_NO_HIP_MEMORY_CACHING=1 step light_nocache 300 python3 bench.py $LIGHT
echo "== done"
