#!/usr/bin/env python3
"""Profile the reference family (UA + HEM + W-cycle + multicolour SGS + coarse
scaling) on one GPU: level sizes, colours per level and the apply's launch
count / time, for rocprofv3 --kernel-trace --stats.

    python bench/prof_ref_family.py [--nrefs 5] [--reps 5] [--coarse-dof 100]
        [--tail-nodes N] [--op-profile]

--op-profile: per (op kind, rows) event time of one eager apply and the
coarse tail's per-op wall-clock stamps (MAMG_OP_PROFILE, MAMG_TAIL_PROFILE;
device.hip dev_time_apply), on stderr.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# per-op event times and the coarse tail's stamps exist in the diagnosis build only
if '--op-profile' in sys.argv or False:
    os.environ.setdefault('MAMG_LIB', os.path.join(ROOT, 'metric-amg-examples_amd', 'libmamg_diag.so'))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nrefs', type=int, default=5)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--coarse-dof', type=int, default=100)
    ap.add_argument('--tail-nodes', type=int, default=None)
    ap.add_argument('--op-profile', action='store_true')
    ap.add_argument('--timeline', action='store_true', help='with --op-profile: every tail op')
    ap.add_argument('--tail-res', type=int, default=None, help='MAMG_TAIL_RES (register-resident tail operators)')
    ap.add_argument('--opt', action='append', default=[], help='NAME=VALUE: a layout switch (mamg_set_option)')
    ap.add_argument('--pcg', action='store_true', help='also the device PCG iterations (rtol 1e-6)')
    args = ap.parse_args()
    import torch
    import metric_amg_examples_amd as M
    if args.tail_nodes is not None:
        M._lib.set_option('MAMG_TAIL_NODES', args.tail_nodes)
    if args.tail_res is not None:
        M._lib.set_option('MAMG_TAIL_RES', args.tail_res)
    for kv in args.opt:
        k, v = kv.split('=', 1)
        M._lib.set_option(k, v)
    n = M.problems.finest_n(3, args.nrefs)
    s = M.problems.bidomain(3, n, 1e6)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup='gpu', AMG_type=1, aggregation_type=5,
                    cycle_type=2, smoother=11, coarse_scaling=1, Schwarz_type=7, coarse_dof=args.coarse_dof,
                    print_level=1)
    print('levels', B.num_levels, flush=True)
    r = torch.as_tensor(M.problems.seeded_rhs(s.N)).cuda()
    z = torch.zeros_like(r)
    B.apply_device(r, z)
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(args.reps):
        B.apply_device(r, z)
    torch.cuda.synchronize()
    print('ms/apply %.3f' % ((time.time() - t) / args.reps * 1e3), flush=True)
    print('znorm %.17g' % float(torch.linalg.norm(z)), flush=True)
    if args.pcg:   # bench.py's PCG (cbc.block ConjGrad, 1e-8), device-resident
        B._Aop = A
        cg = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
        torch.cuda.synchronize()
        t = time.time()
        cg * r
        torch.cuda.synchronize()
        print('pcg niters %d residual %.6e %.3f s' % (len(cg.residuals) - 1, cg.residuals[-1], time.time() - t),
              flush=True)
    if args.op_profile:
        os.environ['MAMG_OP_PROFILE'] = '1'
        os.environ['MAMG_TAIL_PROFILE'] = '2' if args.timeline else '1'
        st = torch.cuda.current_stream()
        ms, _, _ = B.time_apply(r, z, 2, 1, st)
        torch.cuda.synchronize()
        print('eager instrumented ms/apply %.3f' % ms, flush=True)


if __name__ == '__main__':
    main()
