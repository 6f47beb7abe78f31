#!/bin/bash
# Round-6 GPU call B: (1) the round-5 crash case (nrefs=5, 8 virtual ranks,
# reference preset, lockstep apply as one hipGraph) with the instantiation on
# a helper thread sized to the graph and no op cap; (2) the N>1 bench line's
# one-GPU parity check (2 ranks on one GPU, host-staged gloo exchange).
OUT=$(pwd)/gpurun_out/r06b
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -4 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
MAMG_LIB=$(pwd)/metric-amg-examples_amd/libmamg_diag.so step s5_8 600 \
  python -X faulthandler -u bench/dist_rehearsal.py --nrefs 5 --ranks 8 --profile schwarz
step gloo2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --exchange gloo --steps 5 --warmup 2
echo "== done"
