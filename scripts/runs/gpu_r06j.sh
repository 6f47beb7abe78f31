#!/bin/bash
# coarse tail: shader clock vs wall clock during the tail program
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 5 --tail-res 1 --op-profile --timeline > $O/ref_res1.log 2>&1 || { echo "failed"; tail -20 $O/ref_res1.log; exit 1; }
grep -E "ms/apply|mamg tail\]" $O/ref_res1.log
