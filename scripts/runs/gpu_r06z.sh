#!/bin/bash
# final tree, N = 2 (two ranks on the one GPU, host-staged gloo exchange): the bench line with its one-GPU parity check
set -o pipefail
O=$PWD/gpurun_out/r06z; mkdir -p $O
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --exchange gloo --steps 10 --warmup 2 --cpu-sample 0 --compare-profiles 0 > $O/b2.log 2>&1 || { echo "2-rank bench failed"; tail -20 $O/b2.log; exit 1; }
grep '^{' $O/b2.log | tail -1 > $O/b2.json
python3 -c "
import json; d=json.load(open('$O/b2.json'))
print(d['value'], d['n_gpus'], d.get('pcg',{}).get('niters'), json.dumps(d.get('check_1gpu'))[:600])"
