#!/bin/bash
# patch inverse kernels: time of each variant (2 scalar, 3 matrix cores, 4 assembly only, 5 sweep only; diag lib)
set -o pipefail
O=$PWD/gpurun_out/r06r; ROOT=$PWD; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MAMG_LIB=$ROOT/metric-amg-examples_amd/libmamg_diag.so
for v in 2 3 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o p -- python3 $ROOT/bench/prof_patch_setup.py --opt MAMG_PATCH_INV=$v > $O/t$v.log 2>&1 || { echo "v=$v failed"; tail -5 $O/t$v.log; exit 1; }
  echo "v=$v"; grep -h "patch_inv" $O/t$v/*kernel_stats.csv | cut -d, -f1-4 | sed 's/(long.*)"/"/'
done
