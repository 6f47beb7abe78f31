#!/bin/bash
# Round-4 GPU call E14: bench/contig_alias.hip -- do allocations of one kind
# (contiguous / hipMalloc / hipMallocAsync) share memory with other live
# allocations?  Kind masks: 1 contiguous, 2 hipMalloc, 4 hipMallocAsync.
TAG=${1:-r04e14}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 hipcc -O2 --offload-arch=gfx950 bench/contig_alias.hip -o $OUT/contig_alias || exit 1
step() {
  local name=$1; shift
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 150 "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(tail -1 $OUT/$name.txt)" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP ($rc)"; exit $rc; fi
}
for seed in 1234567 987654321 55555; do
  for k in 2 6 4 3 5 7; do
    step k${k}_s$seed $OUT/contig_alias 4000 $k 50 $seed
  done
done
echo "== done"
