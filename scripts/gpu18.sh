source scripts/gpu_run.sh
export TMPDIR=/tmp
step gpu_setup_tests 600 python -u -m pytest tests/test_gpu_setup.py -x -v --timeout 300 --timeout-method thread
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 3 --pcg --compare-host-setup
