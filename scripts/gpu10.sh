source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step variants 900 python bench/variants.py MAMG_SELL=1 MAMG_SELL=0 MAMG_SELL=1,MAMG_SYM_BLOCKS=0
