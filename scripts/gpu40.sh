source scripts/gpu_run.sh
export TMPDIR=/tmp
step bench_2d6 600 python bench.py --dim 2 --nrefs 6 --gamma 1e6 --steps 50 --warmup 5 --pcg
step bench_3d5 600 python bench.py --dim 3 --nrefs 5 --gamma 1e6 --steps 50 --warmup 5 --pcg
