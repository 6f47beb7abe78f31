#!/bin/bash
# Round-5 GPU call Z9: the multi-second setups of the bench's long-lived process
# (one phase of one or two profiles per run): setup temporaries' cache trimmed
# at the end of every setup (default) vs kept for the next (MAMG_TMP_KEEP=1),
# alternating on one box.
OUT=$(pwd)/gpurun_out/r05z9
mkdir -p $OUT
for r in a b; do
  for k in 0 1; do
    MAMG_TMP_KEEP=$k timeout -k 10 400 python -u bench.py --cpu-sample 0 --steps 5 > $OUT/k$k$r.log 2>&1 || exit 1
    tail -1 $OUT/k$k$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('TMP_KEEP=$k', d['value'], d['setup']['wall_s'], [round(p['setup_s'],2) for p in d['pcg_profiles']])"
  done
done
