#!/bin/bash
# long-lived process: patch presets one after another, without and with a pause after each close
set -o pipefail
O=$PWD/gpurun_out/r06v; mkdir -p $O
for pz in 0 5; do
  timeout -k 10 400 python3 -u bench/prof_patch_setup.py --sequence patch,ref,patch,ref --pause $pz > $O/seq_p$pz.log 2>&1 || { echo "seq failed"; tail -5 $O/seq_p$pz.log; exit 1; }
  echo "pause $pz"; grep -o '"profile": "[a-z]*", "setup_s": [0-9.]*\|"close_s": [0-9.]*\|"aggregate": [0-9.]*\|"layout_build": [0-9.]*' $O/seq_p$pz.log | tr '\n' ' '; echo
done
