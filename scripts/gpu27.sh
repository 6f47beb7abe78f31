source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step variants 900 python bench/variants.py --reps 30 MAMG_HALF=1 MAMG_HALF_REMAP=1 MAMG_HALF=0 MAMG_HALF=1
step bench 600 python bench.py --steps 20 --warmup 3
step kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt27 -o kt -- python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-breakdown
step fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "sell2_kernel|bsr2_post|bsr2_kernel" --output-format csv -d $R/gpurun_out/f27 -o f -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
step write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "sell2_kernel|bsr2_post|bsr2_kernel" --output-format csv -d $R/gpurun_out/w27 -o w -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
