source scripts/gpu_run.sh
export TMPDIR=/tmp
export MAMG_BENCH_DEVICE=0
step twoRanksOneGpu 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --nrefs 4 --steps 5 --warmup 2 --pcg
