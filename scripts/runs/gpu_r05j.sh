#!/bin/bash
# Round-5 GPU call J: node patches on N ranks (virtual ranks, two gloo
# processes), then the whole dist test file.
OUT=$(pwd)/gpurun_out/r05j
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step patches 600 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "node_patches or host_exchange"
step dist 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_rings.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
MAMG_LIB=$(pwd)/metric-amg-examples_amd/libmamg_diag.so MAMG_DEBUG_PTRS=1 MAMG_POISON=1 \
  step debugptrs 600 python -u -m pytest tests/test_gpu.py -q -s -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "test_k_kernel_variants or test_half_symmetric_a0_bitwise or test_post_operator_k_equals_merged or test_multiple_handles_and_graph_cache or test_host_apply_after_queued_device_apply"
echo "debug-check reports: $(grep -c 'mamg debug' $OUT/debugptrs.log)" | tee -a $OUT/steps.log
echo "== done"
