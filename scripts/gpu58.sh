source scripts/gpu_run.sh
export TMPDIR=/tmp
step variants 900 python bench/variants.py --reps 40 MAMG_NT=0 MAMG_NT=1 MAMG_NT=0 MAMG_NT=1 MAMG_NT=0 MAMG_NT=1
