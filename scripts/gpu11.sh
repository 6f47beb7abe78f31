source scripts/gpu_run.sh
export TMPDIR=/tmp
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step variants 900 python bench/variants.py MAMG_SELL_POST=0 MAMG_SELL_POST=1
