source scripts/gpu_run.sh
export TMPDIR=/tmp
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step b1a 300 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step b0a 300 env MAMG_PRERESERVE_B_PER_NNZ=0 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step b1b 300 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step b0b 300 env MAMG_PRERESERVE_B_PER_NNZ=0 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
export MAMG_DIST_DRY=1
step dry8 900 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8
