#!/bin/bash
# register-resident coarse tail: parity tests, then the reference family A/B at nrefs=6
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gs.py -x -v --timeout 300 --timeout-method thread > $O/gs.log 2>&1 || { echo "gs tests failed"; tail -30 $O/gs.log; exit 1; }
tail -2 $O/gs.log
for res in 0 1; do
  timeout -k 10 300 python -u bench/prof_ref_family.py --nrefs 6 --reps 10 --tail-res $res --pcg > $O/ref_res$res.log 2>&1 || { echo "ref family res=$res failed"; tail -20 $O/ref_res$res.log; exit 1; }
  grep -E "levels|ms/apply|znorm|pcg" $O/ref_res$res.log
done
