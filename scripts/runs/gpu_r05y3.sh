#!/bin/bash
# Round-5 GPU call Y3: where the first reference-family setup of the bench
# process spends 5 s in its Galerkin phase: the diagnosis build's SpGEMM
# trace (allocations vs products, free HBM) during the bench's profile
# comparison (after: one staging block per device, kept for the process).
OUT=$(pwd)/gpurun_out/r05y4
mkdir -p $OUT
export MAMG_LIB=$(pwd)/metric-amg-examples_amd/libmamg_diag.so MAMG_SPGEMM_TRACE=1
timeout -k 10 600 python -u bench.py --cpu-sample 0 --steps 5 --pcg 1 --compare-profiles 1 > $OUT/b.log 2>&1
echo "rc=$?"
grep -c "mamg spgemm" $OUT/b.log
grep "mamg spgemm" $OUT/b.log | sort -t, -k2 -rn | head -5
awk '/mamg spgemm/ { split($0,a,"allocations "); split(a[2],b," ms"); if (b[1] > 50) print }' $OUT/b.log | head -20
