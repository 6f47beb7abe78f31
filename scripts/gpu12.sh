source scripts/gpu_run.sh
export TMPDIR=/tmp
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step variants 900 python bench/variants.py MAMG_PREFETCH=1 MAMG_PREFETCH=0 MAMG_POST_LANES=4 MAMG_POST_LANES=16 MAMG_SELL=0
