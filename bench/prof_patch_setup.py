#!/usr/bin/env python3
"""Setup of the reference's verbatim preset parameters_metric_schwarz
(src/amg_parameters.py:67-89: UA + HEM + W + SGS + scaling + SCHWARZ_SYMMETRIC
1-rings, run as SCHWARZ_PATCHES) on one GPU: wall time and setup phases, for
rocprofv3 --kernel-trace --stats (which kernels the node-patch layout build
spends its time in).

    python bench/prof_patch_setup.py [--nrefs 6] [--applies 0] [--profile ref|patch]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nrefs', type=int, default=6)
    ap.add_argument('--applies', type=int, default=0)
    ap.add_argument('--profile', choices=('ref', 'patch'), default='ref',
                    help='ref: the verbatim preset; patch: mi355x_patch (node-block Jacobi below level 0)')
    ap.add_argument('--check', type=int, default=0,
                    help='n > 0: compare the first n patch inverses with a float64 numpy inverse')
    ap.add_argument('--opt', action='append', default=[], help='NAME=VALUE: a layout switch (mamg_set_option)')
    ap.add_argument('--pause', type=float, default=0.0, help='--sequence: seconds to wait after each close')
    ap.add_argument('--sequence', default=None,
                    help='comma-separated profiles (ref, patch) set up and closed one after another in this '
                         'process (the bench\'s long-lived process), each timed')
    args = ap.parse_args()
    import torch
    import metric_amg_examples_amd as M
    for kv in args.opt:
        k, v = kv.split('=', 1)
        M._lib.set_option(k, v)
    n = M.problems.finest_n(3, args.nrefs)
    s = M.problems.bidomain(3, n, 1e6)
    A = s.scipy()
    def kw_of(prof):
        if prof == 'ref':
            return dict(AMG_type=1, aggregation_type=5, cycle_type=2, smoother=11, coarse_scaling=1,
                        strong_coupled=0.1, Schwarz_type=6, relaxation=1.2, Schwarz_maxlvl=1)
        return dict(smoother=3, Schwarz_type=6, Schwarz_maxlvl=1)
    if args.sequence:
        for prof in args.sequence.split(','):
            torch.cuda.synchronize()
            t0 = time.time()
            B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup='gpu', **kw_of(prof))
            torch.cuda.synchronize()
            ts = time.time() - t0
            r = torch.as_tensor(M.problems.seeded_rhs(s.N)).cuda()
            z = torch.zeros_like(r)
            ms, _, _ = B.time_apply(r, z, 2, 0, torch.cuda.current_stream())
            print(json.dumps({'profile': prof, 'setup_s': round(ts, 3), 'ms_per_apply': round(ms, 3),
                              'hbm_free_gb': round(torch.cuda.mem_get_info()[0] / 2**30, 1),
                              'phases_ms': {k: round(v, 1) for k, v in B.setup_timings.items()}}), flush=True)
            t0 = time.time()
            B.close()
            torch.cuda.synchronize()
            print(json.dumps({'close_s': round(time.time() - t0, 3)}), flush=True)
            if args.pause:
                time.sleep(args.pause)
        return
    kw = kw_of(args.profile)
    torch.cuda.synchronize()
    t0 = time.time()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup='gpu', **kw)
    torch.cuda.synchronize()
    ts = time.time() - t0
    out = {'nrefs': args.nrefs, 'N': s.N, 'profile': args.profile, 'setup_s': round(ts, 3),
           'phases_ms': {k: round(v, 1) for k, v in B.setup_timings.items()}}
    if args.applies:
        r = torch.as_tensor(M.problems.seeded_rhs(s.N)).cuda()
        z = torch.zeros_like(r)
        ms, _, _ = B.time_apply(r, z, args.applies, 1, torch.cuda.current_stream())
        out['ms_per_apply'] = round(ms, 3)
    print(json.dumps(out), flush=True)
    B.close()


if __name__ == '__main__':
    main()
