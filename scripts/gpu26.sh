source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step gpu_half 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "half or sell_layout"
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step variants 900 python bench/variants.py --reps 30 MAMG_HALF=0 MAMG_HALF=1 MAMG_HALF=1,MAMG_HALF_U=4 MAMG_HALF=1,MAMG_SELL_REMAP=1 MAMG_HALF=0
step bench 600 python bench.py --steps 20 --warmup 3
