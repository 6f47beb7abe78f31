source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_n6 600 python bench.py --steps 20
step prof_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kt3 -o kt -- python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-breakdown
