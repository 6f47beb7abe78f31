source scripts/gpu_run.sh
export TMPDIR=/tmp
step variants 900 python bench/variants.py --reps 40 MAMG_POST_U=4 MAMG_POST_U=6 MAMG_POST_U=4 MAMG_POST_U=6 MAMG_POST_U=4 MAMG_POST_U=6
