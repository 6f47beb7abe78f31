source scripts/gpu_run.sh
export TMPDIR=/tmp
step reh5 300 python -u bench/dist_rehearsal.py --nrefs 5 --ranks 8
step reh6 900 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8
