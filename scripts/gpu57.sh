source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 600 python bench.py
step bench_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt57 -o kt -- python bench.py --cpu-sample 0 --no-breakdown
