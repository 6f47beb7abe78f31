source scripts/gpu_run.sh
nproc > gpurun_out/nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1; rocm-smi > gpurun_out/rocm-smi.txt 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step bench_n5 300 python bench.py --nrefs 5 --steps 10 --cpu-sample 1
step bench_n6 600 python bench.py --steps 20
