source scripts/gpu_run.sh
export TMPDIR=/tmp
step variants 900 python bench/variants.py --reps 40 MAMG_POST_BANDS=0 MAMG_POST_BANDS=1 MAMG_POST_BANDS=0 MAMG_POST_BANDS=1 MAMG_POST_BANDS=0 MAMG_POST_BANDS=1
