source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step micro 400 ./bench/spmv_micro 256 10
step pytest_gpu 900 python -m pytest tests -m gpu -q
step prof_kt 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof_kt -o kt -- python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-breakdown
step prof_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex csr_kernel -T --output-format csv -d $R/gpurun_out/prof_fetch -o f -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
step prof_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex csr_kernel -T --output-format csv -d $R/gpurun_out/prof_write -o w -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
