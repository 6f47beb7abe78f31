source scripts/gpu_run.sh
export TMPDIR=/tmp
step gpu_blocks 600 python -u -m pytest tests/test_gpu_blocks.py -x -v --timeout 300 --timeout-method thread
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step driver_emi3d 600 python -m metric_amg_examples_amd.drivers emi_3d -nrefs 5 -gamma 1e6 -results gpurun_out/results
step driver_bid3d 600 python -m metric_amg_examples_amd.drivers bidomain_3d -nrefs 5 -gamma 1e6 -results gpurun_out/results
