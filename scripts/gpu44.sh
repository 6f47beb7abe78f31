source scripts/gpu_run.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "hsell2_kernel|sell2_kernel" --output-format csv -d $R/gpurun_out/f44 -o f -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
step write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "hsell2_kernel|sell2_kernel" --output-format csv -d $R/gpurun_out/w44 -o w -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-breakdown
step bench_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt44 -o kt -- python bench.py --steps 20 --warmup 3 --cpu-sample 0 --no-breakdown
step bench 600 python bench.py
step bench_pcg 600 python bench.py --steps 20 --warmup 3 --pcg
