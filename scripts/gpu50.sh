source scripts/gpu_run.sh
export TMPDIR=/tmp
step variants 900 python bench/variants.py --reps 40 MAMG_HALF_U=4 MAMG_HALF_U=8 MAMG_HALF_U=4 MAMG_HALF_U=8
