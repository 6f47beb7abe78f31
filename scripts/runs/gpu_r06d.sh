#!/bin/bash
# Round-6 GPU call D: seed-ring Schwarz on N ranks (virtual ranks vs one GPU
# and the oracle, config 4's own call on 8 ranks), the concurrent-setup test
# with the capture lock, the rings / setup / dist suites, and the round-5
# nrefs=6 8-rank reference-preset rehearsal (r05k crashed there).
OUT=$(pwd)/gpurun_out/r06d
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -4 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step rings 600 python -u -m pytest tests/test_gpu_rings.py tests/test_gpu_setup.py -m gpu -v --timeout 300 --timeout-method thread -k "rings or concurrent or cache"
step config4 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -v -s --timeout 500 --timeout-method thread -k "default_rings"
step schwarz8 600 python -X faulthandler -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --profile schwarz
echo "== done"
