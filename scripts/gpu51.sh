source scripts/gpu_run.sh
export TMPDIR=/tmp
step b0a 300 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step b1a 300 env MAMG_PRERESERVE_B_PER_NNZ=20 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step b0b 300 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step b1b 300 env MAMG_PRERESERVE_B_PER_NNZ=20 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step b0c 300 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step b1c 300 env MAMG_PRERESERVE_B_PER_NNZ=20 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
