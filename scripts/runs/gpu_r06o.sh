#!/bin/bash
# coarse tail: image-loaded resident rows; tail tests; reference family timing + PCG
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gs.py -x -v --timeout 300 --timeout-method thread > $O/gs.log 2>&1 || { echo "gs tests failed"; tail -30 $O/gs.log; exit 1; }
tail -1 $O/gs.log
timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 10 --pcg > $O/ref.log 2>&1 || { echo "ref failed"; tail -20 $O/ref.log; exit 1; }
grep -E "ms/apply|znorm|pcg" $O/ref.log
timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 5 --op-profile > $O/ref_prof.log 2>&1 || { echo "ref prof failed"; tail -20 $O/ref_prof.log; exit 1; }
grep -E "^ms/apply|kind 13|program of|empty op|tail\] kind [59]" $O/ref_prof.log
