#!/bin/bash
# Round-6 GPU call C: the GPU suite, smoke and the N = 1 bench line on the
# tree with the option table, the bounded setup cache, the staging lease and
# the graph-instantiation helper (scripts/gpu_check.sh steps).
bash scripts/gpu_check.sh r06c smoke,tests,bench
