#!/bin/bash
# patch inverses with LDS assembly + packed stores: patch tests, then kernel times of v1 (round 5), v2, v3, parts 4/5
set -o pipefail
O=$PWD/gpurun_out/r06s; ROOT=$PWD; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_patch.py -x -v --timeout 300 --timeout-method thread > $O/patch.log 2>&1 || { echo "patch tests failed"; grep -E "FAIL|Error|assert" $O/patch.log | head -20; tail -5 $O/patch.log; exit 1; }
tail -1 $O/patch.log
cd /tmp && export TMPDIR=/tmp
export MAMG_LIB=$ROOT/metric-amg-examples_amd/libmamg_diag.so
for v in 2 3 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o p -- python3 $ROOT/bench/prof_patch_setup.py --opt MAMG_PATCH_INV=$v > $O/t$v.log 2>&1 || { echo "v=$v failed"; tail -5 $O/t$v.log; exit 1; }
  echo "v=$v $(grep -h 'patch_inv' $O/t$v/*kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3)"
done
