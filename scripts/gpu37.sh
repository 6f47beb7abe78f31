source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step setup_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt37 -o kt -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
