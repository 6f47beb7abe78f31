source scripts/gpu_run.sh
export TMPDIR=/tmp
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step variants 900 python bench/variants.py MAMG_SELL_U=8 MAMG_SELL_U=4 MAMG_SELL_U=4,MAMG_SELL_PRE=1 MAMG_SELL_U=8,MAMG_SELL_PRE=1 MAMG_SELL_U=16 MAMG_SELL_U=16,MAMG_SELL_PRE=1 MAMG_SELL_U=8
