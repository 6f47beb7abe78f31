source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step variants 900 python bench/variants.py MAMG_NT=0 MAMG_NT=1 MAMG_NT=1,MAMG_SELL_U=4 MAMG_NT=0
step fetch_nt 600 env MAMG_NT=1 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "sell2_kernel|bsr2_post" --output-format csv -d $R/gpurun_out/f15 -o f -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
