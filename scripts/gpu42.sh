source scripts/gpu_run.sh
export TMPDIR=/tmp
export MAMG_DIST_DRY=1
step dry8 900 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 8
step dry2 600 python -u bench/dist_rehearsal.py --nrefs 6 --ranks 2
