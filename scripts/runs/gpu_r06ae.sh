#!/bin/bash
# Round-6 final checkpoint: smoke, the GPU suite, bench (N=1), kernel trace and the PMC traffic passes of the final tree
bash scripts/gpu_check.sh r06ae smoke,tests,bench,trace,pmc
