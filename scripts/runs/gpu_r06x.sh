#!/bin/bash
# residual kernel occupancy sweep (diag build: dynamic LDS pad caps workgroups per CU), then FETCH for two pads
set -o pipefail
O=$PWD/gpurun_out/r06x; ROOT=$PWD; mkdir -p $O
export MAMG_LIB=$ROOT/metric-amg-examples_amd/libmamg_diag.so
for pad in 0 32768 40960 54000; do
  MAMG_HALF_LDS_PAD=$pad timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --cpu-sample 0 --pcg 0 --compare-profiles 0 --no-breakdown > $O/b$pad.log 2>&1 || { echo "pad $pad failed"; tail -5 $O/b$pad.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('$O/b$pad.log') if l.startswith('{')][-1])
r=[k for k in d['roofline_kernels'] if 'residual' in k['kernel']][0]
print('pad $pad', d['value'], 'resid ms', r['ms_per_launch'])"
done
