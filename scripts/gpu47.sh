source scripts/gpu_run.sh
export TMPDIR=/tmp
step variants 900 python bench/variants.py --reps 40 MAMG_ARENA_GB=0 MAMG_ARENA_GB=24 MAMG_ARENA_GB=0 MAMG_ARENA_GB=24 MAMG_ARENA_GB=0 MAMG_ARENA_GB=24 MAMG_ARENA_GB=0 MAMG_ARENA_GB=24
