#!/bin/bash
# the coarsest dense inverse in the tail's LDS region: tail tests, reference family timing + PCG, per-op stamps
set -o pipefail
O=gpurun_out/r06ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gs.py -x -v --timeout 300 --timeout-method thread > $O/gs.log 2>&1 || { echo "gs tests failed"; grep -E "FAIL|Error" $O/gs.log | head; tail -3 $O/gs.log; exit 1; }
tail -1 $O/gs.log
timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 10 --pcg > $O/ref.log 2>&1 || { echo "ref failed"; tail -20 $O/ref.log; exit 1; }
grep -E "ms/apply|znorm|pcg" $O/ref.log
timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 5 --op-profile > $O/ref_prof.log 2>&1 || { echo "ref prof failed"; tail -20 $O/ref_prof.log; exit 1; }
grep -E "kind 13|program of|tail\] kind [029]" $O/ref_prof.log
