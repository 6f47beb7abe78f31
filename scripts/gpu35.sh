source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "hsell2_kernel|sell2_kernel" --output-format csv -d $R/gpurun_out/f35 -o f -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
step write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "hsell2_kernel|sell2_kernel" --output-format csv -d $R/gpurun_out/w35 -o w -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
step bench_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt35 -o kt -- python bench.py --steps 20 --warmup 3 --cpu-sample 0 --no-breakdown
step bench 600 python bench.py --steps 20 --warmup 3 --pcg
