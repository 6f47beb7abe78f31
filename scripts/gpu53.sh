source scripts/gpu_run.sh
export TMPDIR=/tmp
step c1a 300 env MAMG_PRERESERVE_CONTIG=1 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step c0a 300 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step n0a 300 env MAMG_PRERESERVE_B_PER_NNZ=0 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step c1b 300 env MAMG_PRERESERVE_CONTIG=1 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step c0b 300 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
step n0b 300 env MAMG_PRERESERVE_B_PER_NNZ=0 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --no-breakdown
