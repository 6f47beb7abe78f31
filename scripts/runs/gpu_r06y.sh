#!/bin/bash
# Jacobi headline with the register-resident coarse tail on its smallest levels (diag lib reads MAMG_TAIL_NODES), A/B/A
set -o pipefail
O=$PWD/gpurun_out/r06y; ROOT=$PWD; mkdir -p $O
export MAMG_LIB=$ROOT/metric-amg-examples_amd/libmamg_diag.so
for tn in 0 100 0 100; do
  MAMG_TAIL_NODES=$tn timeout -k 10 300 python3 -u bench.py --steps 40 --warmup 5 --cpu-sample 0 --pcg 0 --compare-profiles 0 --no-breakdown > $O/b$tn.log 2>&1 || { echo "tn $tn failed"; tail -5 $O/b$tn.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/b$tn.log') if l.startswith('{')][-1])
print('tail nodes $tn', d['value'], d['ms_per_step'], d['graph_ms_per_step'])"
done
