source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step bench 600 python bench.py --steps 20 --warmup 3
step bench_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt6 -o kt -- python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-breakdown
