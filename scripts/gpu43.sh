source scripts/gpu_run.sh
export TMPDIR=/tmp
step dist_tests 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread
export MAMG_DIST_DRY=1
step dry8 900 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8
