#!/bin/bash
# matrix-core patch inverses: patch tests, then the verbatim preset's setup trace (v3 default vs v2)
set -o pipefail
O=$PWD/gpurun_out/r06q; ROOT=$PWD; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_patch.py -x -v --timeout 300 --timeout-method thread > $O/patch.log 2>&1 || { echo "patch tests failed"; grep -E "FAIL|Error|assert" $O/patch.log | head -20; tail -5 $O/patch.log; exit 1; }
tail -1 $O/patch.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace3 -o p -- python3 $ROOT/bench/prof_patch_setup.py > $O/trace3.log 2>&1 || { echo "trace3 failed"; tail -5 $O/trace3.log; exit 1; }
tail -4 $O/trace3.log
grep -h "patch_inv" $O/trace3/*kernel_stats.csv | cut -c1-40,200-400 || true
