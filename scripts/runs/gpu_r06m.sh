#!/bin/bash
# coarse tail: resident rows without predicates; program in LDS vs scalar loads
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
for pl in 0; do
  timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 5 --tail-res 1 --opt MAMG_TAIL_PROG_LDS=$pl --op-profile --timeline > $O/pl$pl.log 2>&1 || { echo "pl=$pl failed"; tail -20 $O/pl$pl.log; exit 1; }
  grep -E "ms/apply|empty ops|program of|kind 13" $O/pl$pl.log
done
