source scripts/gpu_run.sh
export TMPDIR=/tmp
step setup_tests 600 python -u -m pytest tests/test_gpu_setup.py -x -q --timeout 300 --timeout-method thread
step bench 600 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-breakdown
