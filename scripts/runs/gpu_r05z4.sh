#!/bin/bash
# Round-5 GPU call Z4: setup staging with RS_BATCH loads in flight and the
# grid-stride sym check: the staging micro, the setup/layout bitwise tests,
# bench setup phases (twice) and a kernel trace of the bench for per-launch
# setup kernel times.
OUT=$(pwd)/gpurun_out/r05z4
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
step micro 120 ./bench/setup_stage_micro.bin
cat $OUT/micro.log
step t_setup 400 python -u -m pytest tests/test_gpu_setup.py -x -q --timeout 200 --timeout-method thread
step b1 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown
step b2 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown
for b in b1 b2; do tail -1 $OUT/$b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['setup']
print('$b', d['value'], s['wall_s'], s['phases_ms'])"; done
cd /tmp && step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench \
    -- python3 $ROOT/bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-breakdown --pcg 0 --compare-profiles 0; cd $ROOT
echo "== done"
