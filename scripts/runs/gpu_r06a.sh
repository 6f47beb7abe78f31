#!/bin/bash
# Round-6 GPU call A: the graph-capture SIGSEGV of round 5 (r05l/s5_8.log:
# nrefs=5, 8 virtual ranks, reference preset, mamg_dist_virtual_apply_graph),
# run once under the diagnosis build's SIGSEGV tracer with the op cap lifted.
OUT=$(pwd)/gpurun_out/r06a
mkdir -p $OUT
echo "stack limit: $(ulimit -s) KiB (hard $(ulimit -Hs))" > $OUT/env.txt
MAMG_LIB=$(pwd)/metric-amg-examples_amd/libmamg_diag.so MAMG_GRAPH_MAX_OPS=100000000 \
  timeout -k 10 600 python -X faulthandler -u bench/dist_rehearsal.py --nrefs 5 --ranks 8 --profile schwarz \
  > $OUT/s5_8.log 2>&1
rc=$?
echo "rc=$rc" >> $OUT/env.txt
tail -60 $OUT/s5_8.log
exit $rc
