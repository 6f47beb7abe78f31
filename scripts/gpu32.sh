source scripts/gpu_run.sh
export TMPDIR=/tmp
step band_test 300 python -u -m pytest tests/test_gpu.py -k "band_schedule or half_symmetric" -x -q --timeout 200 --timeout-method thread
step variants 900 python bench/variants.py --reps 30 MAMG_HALF_BANDS=0 MAMG_HALF_BANDS=1 MAMG_HALF_BANDS=2 MAMG_HALF_BANDS=4 MAMG_HALF_BANDS=8 MAMG_HALF_BANDS=0
