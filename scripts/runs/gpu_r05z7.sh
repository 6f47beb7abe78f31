#!/bin/bash
# Round-5 GPU call Z7: is the level-0 K time of the last runs (all four K value
# regions ~1.41 ms) the box or the MIS-2 staging?  Alternating on one box.
OUT=$(pwd)/gpurun_out/r05z7
mkdir -p $OUT
for r in a b; do
  for m in 1 0; do
    MAMG_MIS_STAGED=$m timeout -k 10 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 10 --no-breakdown > $OUT/m$m$r.log 2>&1 || exit 1
    tail -1 $OUT/m$m$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['setup']
print('MIS_STAGED=$m', d['value'], d['k_region'], [k['ms_per_launch'] for k in d['roofline_kernels']], s['wall_s'], s['phases_ms']['aggregate'])"
  done
done
