source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step calib_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex calib --output-format csv -d $R/gpurun_out/cal_f -o f -- ./bench/spmv_micro calib 2
step bsr_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex bsr2_kernel --output-format csv -d $R/gpurun_out/bsr_f -o f -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
step bsr_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex bsr2_kernel --output-format csv -d $R/gpurun_out/bsr_w -o w -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
step bsr_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bsr_kt -o kt -- python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-breakdown
