#!/bin/bash
# Round-4 GPU call B: seed rings after the ordering fix, the restriction band
# schedule and the coarse-tail rework (parity + A/B), one bench line.
#   gpurun --timeout 1200 -- bash scripts/gpu_r04b.sh TAG
TAG=${1:-r04b}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
run() {   # run <name> <timeout> <cmd...>; stop on anything but pass/fail
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP ($rc)"; exit $rc; fi
}
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread"
run quick 400 $PYT tests/test_gpu.py -k "band or tail or k_kernel or multiple_handles or graph_cache"
run rings 400 $PYT tests/test_gpu_rings.py
run bench 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 --pcg 0 --compare-profiles 0
tail -1 $OUT/bench.txt > $OUT/bench.json
MAMG_R_BANDS=0 run bench_rb0 200 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 --pcg 0 --compare-profiles 0
MAMG_R_BANDS=2 run bench_rb2 200 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 --pcg 0 --compare-profiles 0
run ref_new 240 python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 1024 --op-profile
MAMG_LIB=$(pwd)/ab/libmamg_r04base.so run ref_base 240 python -u bench/prof_ref_family.py --nrefs 6 --tail-nodes 1024 --op-profile
echo "== done"
