source scripts/gpu_run.sh
export TMPDIR=/tmp
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 600 python bench.py
