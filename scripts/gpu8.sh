source scripts/gpu_run.sh
export TMPDIR=/tmp
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step variants 900 python bench/variants.py MAMG_XCD_REMAP=1 MAMG_XCD_REMAP=1,MAMG_SYM_BLOCKS=0 MAMG_XCD_REMAP=0 MAMG_XCD_REMAP=2
