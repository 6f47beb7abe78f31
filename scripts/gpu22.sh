source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step gpu_tests 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread
step variants 900 python bench/variants.py --reps 30 MAMG_POST_K=0 MAMG_POST_K=1 MAMG_POST_K=1,MAMG_POST_LANES=4 MAMG_POST_K=1,MAMG_POST_LANES=16 MAMG_POST_K=1,MAMG_SELL_POST=1,MAMG_POST_U=4 MAMG_POST_K=1,MAMG_SELL_POST=1,MAMG_POST_U=8 MAMG_POST_K=1,MAMG_POST_LANES=8,MAMG_XCD_REMAP=2
