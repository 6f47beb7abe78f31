#!/bin/bash
# Round-5 GPU call N: A/B of the restriction's first-sweep epilogue with the
# W block hoisted (MAMG_FUSE_RBD 1 all levels / 2 below level 1 / 0 off),
# alternating, then its bitwise test.
OUT=$(pwd)/gpurun_out/r05n
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -1 "$OUT/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step t_fuse 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "restriction_first_sweep"
B="python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0"
for k in a b c; do
  MAMG_FUSE_RBD=1 step f1$k 300 $B
  MAMG_FUSE_RBD=2 step f2$k 300 $B
  MAMG_FUSE_RBD=0 step f0$k 300 $B
done
echo "== done"
