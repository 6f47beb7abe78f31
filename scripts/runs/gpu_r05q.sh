#!/bin/bash
# Round-5 GPU call Q: wave-per-node CSR -> BSR2 conversion (and SA reusing the
# smoother's node inverses when every node is joined): bitwise tests, the GPU
# setup / dist files, then setup timings with MAMG_CSR2BSR 1 / 0 alternating
# and a kernel trace of one bench setup.
OUT=$(pwd)/gpurun_out/r05q
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step t_conv 300 python -u -m pytest tests/test_gpu_setup.py -x -v --timeout 120 --timeout-method thread -k "csr2bsr"
step t_setup 600 python -u -m pytest tests/test_gpu_setup.py tests/test_gpu_dist.py tests/test_gpu_patch.py -x -q --timeout 200 --timeout-method thread
B="python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown"
for k in a b; do
  step c1$k 300 $B
  MAMG_CSR2BSR=0 step c0$k 300 $B
done
ROOT=$(pwd)
cd /tmp && step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench \
  -- python3 $ROOT/bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-breakdown --pcg 0 --compare-profiles 0
echo "== done"
