# A/B of environment knobs on the default bench workload (one process per
# configuration, short runs); summary lines in gpurun_out/$TAG/summary.txt
#   [BENCH_ARGS="--dim 2"] bash scripts/ab_env.sh TAG "CFG1" "CFG2" ...   (CFG = space-separated VAR=value, or X=0 for the default)
TAG=$1; shift
mkdir -p gpurun_out/$TAG
L="--steps 30 --warmup 3 --cpu-sample 0 --pcg 0 --compare-profiles 0 ${BENCH_ARGS:-}"
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python -u bench.py $L > gpurun_out/$TAG/run.log 2>&1 || exit 1
  python3 -c "
import json,sys;d=json.loads(open('gpurun_out/$TAG/run.log').read().strip().split('\n')[-1]);b=d['breakdown']
print('$cfg', d['value'], d['ms_per_step'], 'K', d['roofline']['ms_per_launch'], 'resid', b['L0_resid']['ms'], 'R', b['L0_restrict']['ms'], 'bd2', b['L0_smoother']['ms'], 'coarse', b['coarse_levels']['ms'], 'inst', b['instrumented_ms_per_apply'])" >> gpurun_out/$TAG/summary.txt
done
