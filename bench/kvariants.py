#!/usr/bin/env python3
"""A/B the level-0 K and residual kernel variants (MAMG_K_VARIANT,
MAMG_R_VARIANT, MAMG_K_LAYOUT; device.hip launch_kvariant / launch_half_u) on
ONE upload of the bidomain_3d hierarchy, so every variant reads the same
physical placement of the operators.

    python bench/kvariants.py [--nrefs 6] [--reps 20] [--rounds 3] k0 k1 k0r1 k0s

A variant is a word of k<K variant>, r<residual variant>, q<restriction
variant> and s / t (K values split into two streams globally / inside each
slot row; default one block per slot).

Variants are timed round-robin (`rounds` times each) with mamg_time_apply
mode 0 (HIP events around the level-0 residual and K launches of every
apply).  One JSON line per (round, variant): K ms, residual ms, ms per apply,
and the apply's relative difference from variant 0 on the same r.
"""
import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nrefs', type=int, default=6)
    ap.add_argument('--gamma', type=float, default=1e6)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('variants', nargs='*', default=['k0', 'k1', 'k2', 'k0r1'])
    args = ap.parse_args()
    import torch
    import metric_amg_examples_amd as M
    n = M.problems.finest_n(3, args.nrefs)
    s = M.problems.bidomain(3, n, args.gamma)
    B = M.MetricAMG(s.scipy(), s.W, idofs=s.idofs, setup='gpu', num_functions=2)
    del s
    N = B.shape[0]
    r = torch.as_tensor(M.problems.seeded_rhs(N)).cuda()
    z = torch.zeros_like(r)
    stream = torch.cuda.current_stream()
    print(json.dumps({'levels': B.num_levels, 'format0': B.level_format(0)}), flush=True)
    zref = None
    for rnd in range(args.rounds):
        for v in args.variants:
            tok = dict(re.findall(r'([krq])(\d+)', v))
            os.environ['MAMG_K_VARIANT'] = tok.get('k', '0')
            os.environ['MAMG_R_VARIANT'] = tok.get('r', '0')
            os.environ['MAMG_RR_VARIANT'] = tok.get('q', '0')
            os.environ['MAMG_K_LAYOUT'] = 'split' if v.endswith('s') else 'split2' if v.endswith('t') else 'block'
            B.time_apply(r, z, 3, 0, stream)                       # warm
            _, cms, _ = B.time_apply(r, z, 5, 1, stream)           # every launch timed: class ms
            ms, kms, _ = B.time_apply(r, z, args.reps, 0, stream)
            torch.cuda.synchronize()
            zc = z.clone()
            if zref is None:
                zref = zc
            diff = float(torch.linalg.norm(zc - zref) / torch.linalg.norm(zref))
            print(json.dumps({'round': rnd, 'variant': v, 'K_ms': round(kms[1], 4),
                              'resid_ms': round(kms[0], 4), 'ms_per_apply': round(ms, 4),
                              'restrict_ms': round(cms[3], 4), 'bd_ms': round(cms[2], 4),
                              'coarse_ms': round(cms[5] + cms[6], 4),
                              'rel_diff_vs_first': diff}), flush=True)
    B.close()


if __name__ == '__main__':
    main()
