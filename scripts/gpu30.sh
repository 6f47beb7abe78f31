source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step gpu_dist 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 600 python bench.py --steps 20 --warmup 3 --pcg
