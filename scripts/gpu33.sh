source scripts/gpu_run.sh
export TMPDIR=/tmp
step variants 900 python bench/variants.py --reps 30 MAMG_POST_REMAP=0 MAMG_POST_REMAP=1 MAMG_POST_REMAP=0 MAMG_POST_REMAP=1 MAMG_POST_REMAP=1,MAMG_POST_U=8
