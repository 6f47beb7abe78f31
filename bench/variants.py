#!/usr/bin/env python3
"""A/B the device tuning knobs on one host hierarchy (bidomain_3d nrefs=6).

    python bench/variants.py [--nrefs 6] [--reps 20] VAR=VAL,VAR=VAL ...

Each argument is one variant: environment knobs read at upload
(MAMG_HALF, MAMG_HALF_BANDS, MAMG_POST_K) plus optional parameter overrides given as
p.<name>=<int> (e.g. p.post_fusion=0).  The setup runs once; every variant
re-uploads it, runs `reps` graph applies (ms per apply) and one instrumented
pass (per-class kernel ms).  One JSON line per variant.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CLASS_NAMES = ['L0_resid', 'L0_smooth_spmv', 'L0_smoother', 'L0_restrict', 'L0_prolong',
               'coarse_levels', 'coarsest_dense', 'misc']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nrefs', type=int, default=6)
    ap.add_argument('--gamma', type=float, default=1e6)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('variants', nargs='*', default=['MAMG_HALF=1'])
    args = ap.parse_args()
    import torch
    import metric_amg_examples_amd as M
    n = M.problems.finest_n(3, args.nrefs)
    s = M.problems.bidomain(3, n, args.gamma)
    H = M.HostHierarchy(s, idofs=s.idofs, num_functions=2)
    r = torch.as_tensor(M.problems.seeded_rhs(s.N)).cuda()
    z = torch.zeros_like(r)
    zref = None
    stream = torch.cuda.current_stream()
    for v in args.variants:
        env = {}
        for kv in v.split(','):
            k, val = kv.split('=')
            env[k] = val
        saved = {}
        for k, val in env.items():
            if k.startswith('p.'):
                saved[k] = getattr(H.params, k[2:])
                setattr(H.params, k[2:], int(val))
            else:
                os.environ[k] = val
        B = M.MetricAMG.from_host(H, s.W)
        for _ in range(3):
            B.apply_device(r, z, stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.reps):
            B.apply_device(r, z, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        _, kms, cb = B.time_apply(r, z, 5, 1, stream)
        zc = z.clone()
        diff = None if zref is None else float(torch.linalg.norm(zc - zref) / torch.linalg.norm(zref))
        if zref is None:
            zref = zc
        print(json.dumps({'variant': v, 'ms_per_apply': round(ms, 4), 'applies_per_s': round(1e3 / ms, 2),
                          'rel_diff_vs_first': diff,
                          'classes': {nm: [round(kms[i], 4), round(cb[i] / 1e9 / (kms[i] * 1e-3), 1)
                                           if kms[i] > 0 else None] for i, nm in enumerate(CLASS_NAMES)}}),
              flush=True)
        B.close()
        for k, val in env.items():
            if k.startswith('p.'):
                setattr(H.params, k[2:], saved[k])
            else:
                del os.environ[k]
    H.close()


if __name__ == '__main__':
    main()
