#!/bin/bash
# Round-6 GPU call G: checkpoint of the tree -- smoke, the GPU suite, the
# N = 1 bench line, its kernel trace and the PMC passes (traffic.json for
# this device.hip).
bash scripts/gpu_check.sh r06g smoke,tests,bench,trace,pmc
