source scripts/gpu_run.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_n6 600 python bench.py --steps 20
