#!/bin/bash
# Round-5 GPU call Z8: half_meta reduced per workgroup (one atomic per counter per workgroup);
# layout tests, bench setup phases, kernel trace.
OUT=$(pwd)/gpurun_out/r05z8
ROOT=$(pwd)
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step t_setup 500 python -u -m pytest tests/test_gpu_setup.py tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "setup or bsr or csr or layout or sym or half"
step b1 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown
step b2 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown
for b in b1 b2; do tail -1 $OUT/$b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['setup']
print('$b', d['value'], s['wall_s'], s['phases_ms'])"; done
cd /tmp && step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench \
    -- python3 $ROOT/bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-breakdown --pcg 0 --compare-profiles 0; cd $ROOT
echo "== done"
