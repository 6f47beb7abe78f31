#!/bin/bash
# Round-5 GPU call M: the coarse first sweep in the restriction's epilogue
# (EPI_YBD) and level 0's K split around the coarse-e halo (multi-GPU);
# their bitwise tests, the GPU suite's dist file, and a bench A/B of
# MAMG_FUSE_RBD (alternating).  Stops at the first crash.
OUT=$(pwd)/gpurun_out/r05m
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step t_fuse 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "restriction_first_sweep or post_fusion or half_band or post_operator"
step t_dist 600 python -u -m pytest tests/test_gpu_dist.py -x -v -s --timeout 200 --timeout-method thread
step b1 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0
MAMG_FUSE_RBD=0 step b0 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0
step b1b 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0
MAMG_FUSE_RBD=0 step b0b 300 python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0
step dist8 600 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8 --source device
echo "== done"
