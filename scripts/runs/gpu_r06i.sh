#!/bin/bash
# register-resident coarse tail: per-op stamps of the tail program, res 0 / 1
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
for res in 0 1; do
  timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 5 --tail-res $res --op-profile --timeline > $O/ref_res$res.log 2>&1 || { echo "res=$res failed"; tail -20 $O/ref_res$res.log; exit 1; }
  grep -E "levels|ms/apply|mamg tail\]" $O/ref_res$res.log
done
