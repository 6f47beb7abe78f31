#!/bin/bash
# reference family: lanes per row of the launched colour steps on levels 5-7 (diag override), A/B
set -o pipefail
O=gpurun_out/r06ad; mkdir -p $O
export MAMG_LIB=$PWD/metric-amg-examples_amd/libmamg_diag.so
for vl in 0 4 8 16 32; do
  MAMG_GS_LANES=$vl timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 10 > $O/vl$vl.log 2>&1 || { echo "vl $vl failed"; tail -5 $O/vl$vl.log; exit 1; }
  echo "vl $vl $(grep -E '^ms/apply|znorm' $O/vl$vl.log | tr '\n' ' ')"
done
