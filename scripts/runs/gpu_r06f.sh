#!/bin/bash
# Round-6 GPU call F: the two-patches-per-wave patch inverse kernel -- its
# bitwise test against the round-5 kernel, the patch / ring suites, and the
# patch presets' setup in a kernel trace (patch_inv2_kernel vs
# patch_inv_kernel: MAMG_PATCH_INV=1 in the second trace).
OUT=$(pwd)/gpurun_out/r06f
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_gpu_patch.py tests/test_gpu_dist.py -m gpu -x -v --timeout 300 --timeout-method thread -k "patch"
cd /tmp
step trace2 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace2 -o p -- python3 $ROOT/bench/prof_patch_setup.py
MAMG_LIB=$ROOT/metric-amg-examples_amd/libmamg_diag.so MAMG_PATCH_INV=1 step trace1 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o p -- python3 $ROOT/bench/prof_patch_setup.py
cd $ROOT
echo "== done"
