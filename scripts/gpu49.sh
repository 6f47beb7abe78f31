source scripts/gpu_run.sh
export TMPDIR=/tmp
step variants 900 python bench/variants.py --reps 40 MAMG_R_LANES=0 MAMG_R_LANES=32 MAMG_R_LANES=16 MAMG_A1_LANES=16 MAMG_A1_LANES=64 MAMG_A1_LANES=8 MAMG_R_LANES=0
