#!/bin/bash
# the patch presets set up one after another in one process (the bench's long-lived process): patch, ref, ref
set -o pipefail
O=$PWD/gpurun_out/r06u; ROOT=$PWD; mkdir -p $O
timeout -k 10 400 python3 -u bench/prof_patch_setup.py --sequence patch,ref,ref > $O/seq3.log 2>&1 || { echo "seq failed"; tail -5 $O/seq3.log; exit 1; }
grep profile $O/seq3.log | cut -c1-330
timeout -k 10 400 python3 -u bench/prof_patch_setup.py --sequence patch,ref --opt MAMG_PATCH_INV=2 > $O/seq2.log 2>&1 || { echo "seq2 failed"; tail -5 $O/seq2.log; exit 1; }
grep profile $O/seq2.log | cut -c1-330
