source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step variants 900 python bench/variants.py MAMG_SYM_BLOCKS=1 MAMG_SYM_BLOCKS=0
step fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex bsr2 --output-format csv -d $R/gpurun_out/f9 -o f -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
step write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex bsr2 --output-format csv -d $R/gpurun_out/w9 -o w -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
