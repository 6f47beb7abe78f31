source scripts/gpu_run.sh
export TMPDIR=/tmp
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step variants 900 python bench/variants.py --reps 40 MAMG_SELL_SPLIT=1 MAMG_SELL_SPLIT=0 MAMG_SELL_SPLIT=1 MAMG_SELL_SPLIT=0 MAMG_SELL_SPLIT=1 MAMG_SELL_SPLIT=0
