#!/bin/bash
# final tree: the reference preset on 8 virtual ranks (nrefs=5 and 6), graph vs eager and vs one GPU
set -o pipefail
O=$PWD/gpurun_out/r06af; mkdir -p $O
for nr in 5 6; do
  timeout -k 10 600 python -X faulthandler -u bench/dist_rehearsal.py --nrefs $nr --ranks 8 --profile schwarz > $O/s${nr}_8.log 2>&1 || { echo "nrefs $nr failed"; tail -20 $O/s${nr}_8.log; exit 1; }
  grep '^{' $O/s${nr}_8.log | tail -1 > $O/s${nr}_8.json
  python3 -c "
import json; d=json.load(open('$O/s${nr}_8.json'))
print('nrefs $nr', {k: d[k] for k in d if 'graph' in k or 'rel' in k or 'iters' in k or 'ms' in k})" | cut -c1-600
done
