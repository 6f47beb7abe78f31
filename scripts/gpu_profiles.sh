#!/bin/bash
# Compare cycle profiles at the north-star size: applies/s, PCG iterations and
# time to solution.  Usage (GPU box): bash scripts/gpu_profiles.sh [nrefs]
set -o pipefail
mkdir -p gpurun_out
NR=${1:-6}
export TMPDIR=/tmp
for prof in "jacobi 0 V" "sgs 0 V" "sgs 1 V" "gs 0 V" "sgs 1 W"; do
  set -- $prof
  tag="${1}_s${2}_${3}_n${NR}"
  echo "== $tag"
  timeout -k 10 300 python bench.py --nrefs $NR --steps 10 --warmup 2 --cpu-sample 0 --no-breakdown --pcg \
      --smoother $1 --scaling $2 --cycle $3 > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err || { echo "FAIL $tag rc=$?"; tail -5 gpurun_out/prof_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/prof_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['pcg'], d['setup'].get('wall_s'))"
done
