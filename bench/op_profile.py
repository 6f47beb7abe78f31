#!/usr/bin/env python3
"""Per-(op kind, rows) event time of one eager apply (MAMG_OP_PROFILE,
device.hip dev_time_apply) for a smoother profile at nrefs N, on stderr.

    python bench/op_profile.py [--nrefs 6] [--profile jacobi|sgs|ref_family] [--reps 5]

Op kinds: 0 CSR, 1 SCALE, 2 GEMV, 3 AXPY, 4 BSR, 5 BD, 6 POST, 7 ILV, 8 GS,
9 ZERO, 10 DOT2, 11 CSCALE, 12 PATCH, 13 TAIL (device.hip OpKind); rows =
the operator's node rows (vector ops: their length).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# per-op event times (MAMG_OP_PROFILE) exist in the diagnosis build only
os.environ.setdefault('MAMG_LIB', os.path.join(ROOT, 'metric-amg-examples_amd', 'libmamg_diag.so'))
sys.path.insert(0, ROOT)

PROFILES = {
    'jacobi': dict(),
    'sgs': dict(smoother=11, coarse_scaling=1, Schwarz_type=7),
    'ref_family': dict(AMG_type=1, aggregation_type=5, cycle_type=2, smoother=11, coarse_scaling=1,
                       Schwarz_type=7),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nrefs', type=int, default=6)
    ap.add_argument('--profile', default='jacobi', choices=sorted(PROFILES))
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    import torch
    import metric_amg_examples_amd as M
    n = M.problems.finest_n(3, args.nrefs)
    s = M.problems.bidomain(3, n, 1e6)
    B = M.MetricAMG(s.scipy(), s.W, idofs=s.idofs, num_functions=2, setup='gpu', **PROFILES[args.profile])
    r = torch.as_tensor(M.problems.seeded_rhs(s.N)).cuda()
    z = torch.zeros_like(r)
    st = torch.cuda.current_stream()
    B.time_apply(r, z, 3, 0, st)
    ms, _, _ = B.time_apply(r, z, args.reps, 0, st)
    print('eager ms/apply %.4f' % ms, flush=True)
    os.environ['MAMG_OP_PROFILE'] = '1'
    ms, _, _ = B.time_apply(r, z, args.reps, 1, st)
    torch.cuda.synchronize()
    print('instrumented ms/apply %.4f' % ms, flush=True)


if __name__ == '__main__':
    main()
