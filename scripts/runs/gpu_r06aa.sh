#!/bin/bash
# 16-bit K columns on the multi-GPU K (per-slice fallback for ghost slices): tests, then 8 virtual ranks dry A/B
set -o pipefail
O=$PWD/gpurun_out/r06aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -k "col16 or dist or virtual or rank" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 0 1 0 1; do
  MAMG_DIST_TEST=dry MAMG_K_COL16=$c timeout -k 10 600 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --source device > $O/dry$c.log 2>&1 || { echo "dry $c failed"; tail -5 $O/dry$c.log; exit 1; }
  echo "col16=$c $(grep -E 'ms|compute' $O/dry$c.log | tail -3 | tr '\n' ' ' | cut -c1-400)"
done
