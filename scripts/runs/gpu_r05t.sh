#!/bin/bash
# Round-5 GPU call S: sharded single-word counters (MIS-2 keys, HEM, rho):
# setup tests, then bench setup timings (3 runs) and a kernel trace.
OUT=$(pwd)/gpurun_out/r05t
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
step t_setup 600 python -u -m pytest tests/test_gpu_setup.py tests/test_gpu_gs.py tests/test_gpu_blocks.py tests/test_gpu_rings.py -x -q --timeout 200 --timeout-method thread
B="python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown"
for k in a b c; do step w$k 300 $B; done
ROOT=$(pwd)
cd /tmp && step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench \
  -- python3 $ROOT/bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-breakdown --pcg 0 --compare-profiles 0
echo "== done"
