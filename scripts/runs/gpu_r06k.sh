#!/bin/bash
# coarse tail: SQ counters of the tail kernel (register-resident rows on)
set -o pipefail
O=$PWD/gpurun_out/r06k; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --output-format csv -d $O/p1 -o ref -- python3 $GRAFT_REPO_ROOT/bench/prof_ref_family.py --nrefs 6 --reps 1 --tail-res 1 > $O/p1.log 2>&1 || { echo p1 failed; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU --output-format csv -d $O/p2 -o ref -- python3 $GRAFT_REPO_ROOT/bench/prof_ref_family.py --nrefs 6 --reps 1 --tail-res 1 > $O/p2.log 2>&1 || { echo p2 failed; tail -5 $O/p2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for p in ('p1', 'p2'):
    f = glob.glob('/root/repo/gpurun_out/r06k/%s/**/*counter_collection.csv' % p, recursive=True)
    if not f: print(p, 'no csv'); continue
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        if 'tail_kernel' not in r['Kernel_Name']: continue
        acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
    for k in sorted(acc): print(p, k, 'per launch %.0f' % (acc[k] / max(1, n[k])), 'launches', n[k])
PY
