source scripts/gpu_run.sh
export TMPDIR=/tmp
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step bench 600 python bench.py --steps 20 --warmup 3
