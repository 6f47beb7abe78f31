#!/bin/bash
# Round-4 GPU call E15: bench/contig_alias.hip with larger sizes -- contiguous
# allocations alone / with hipMalloc, up to 256 MiB; hipMallocAsync alone.
TAG=${1:-r04e15}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 hipcc -O2 --offload-arch=gfx950 bench/contig_alias.hip -o $OUT/contig_alias || exit 1
step() {
  local name=$1; shift
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 200 "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc: $(tail -1 $OUT/$name.txt)" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP ($rc)"; exit $rc; fi
}
for seed in 1234567 987654321; do
  step k1_s${seed}_m11 $OUT/contig_alias 4000 1 50 $seed 11
  step k1_s${seed}_m16 $OUT/contig_alias 1500 1 50 $seed 16
  step k3_s${seed}_m16 $OUT/contig_alias 1500 3 50 $seed 16
  step k2_s${seed}_m16 $OUT/contig_alias 1500 2 50 $seed 16
  step k4_s${seed}_m16 $OUT/contig_alias 1500 4 50 $seed 16
  step k4_s${seed}_m8 $OUT/contig_alias 4000 4 50 $seed 8
done
echo "== done"
