#!/bin/bash
# coarse tail from level 7 (1328 nodes) vs level 8, register-resident rows
set -o pipefail
O=gpurun_out/r06p; mkdir -p $O
for tn in 2000 1024; do
  timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 5 --tail-nodes $tn --op-profile > $O/tn$tn.log 2>&1 || { echo "tn=$tn failed"; tail -20 $O/tn$tn.log; exit 1; }
  echo "tail nodes $tn"; grep -E "^ms/apply|kind 13|program of" $O/tn$tn.log
done
