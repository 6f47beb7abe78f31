#!/usr/bin/env python3
"""A/B of the coarse tail (MAMG_TAIL_NODES: the first level with at most that
many node rows and everything below run by one workgroup, device.hip
tail_kernel) on the bidomain_3d hierarchy, per smoother profile.

    python bench/tail_ab.py [--nrefs 6] [--reps 10] [--nodes 0,4096,16384]

One JSON line per (profile, nodes): ms per apply (eager, mamg_time_apply) and
the coarse-level class ms.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PROFILES = {
    'jacobi': dict(),
    'sgs_w_scaling': dict(smoother=11, coarse_scaling=1, cycle_type=2, Schwarz_type=7),
    'ref_family': dict(AMG_type=1, aggregation_type=5, cycle_type=2, smoother=11, coarse_scaling=1,
                       Schwarz_type=7),
    'ref_family_cd2048': dict(AMG_type=1, aggregation_type=5, cycle_type=2, smoother=11, coarse_scaling=1,
                              Schwarz_type=7, coarse_dof=2048),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nrefs', type=int, default=6)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--nodes', default='0,4096,16384')
    ap.add_argument('--profiles', default=','.join(PROFILES))
    args = ap.parse_args()
    import torch
    import metric_amg_examples_amd as M
    n = M.problems.finest_n(3, args.nrefs)
    s = M.problems.bidomain(3, n, 1e6)
    A = s.scipy()
    r = torch.as_tensor(M.problems.seeded_rhs(s.N)).cuda()
    z = torch.zeros_like(r)
    st = torch.cuda.current_stream()
    for prof in args.profiles.split(','):
        zref = None
        for nodes in args.nodes.split(','):
            os.environ['MAMG_TAIL_NODES'] = nodes
            B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup='gpu', **PROFILES[prof])
            B.time_apply(r, z, 2, 0, st)
            ms, _, _ = B.time_apply(r, z, args.reps, 0, st)
            _, kms, _ = B.time_apply(r, z, 2, 1, st)
            torch.cuda.synchronize()
            zc = z.clone()
            if zref is None:
                zref = zc
            print(json.dumps({'profile': prof, 'tail_nodes': int(nodes), 'levels': B.num_levels,
                              'ms_per_apply': round(ms, 3), 'coarse_ms': round(kms[5] + kms[6] + kms[7], 3),
                              'rel_diff_vs_first': float(torch.linalg.norm(zc - zref) / torch.linalg.norm(zref))}),
                  flush=True)
            B.close()
            del B


if __name__ == '__main__':
    main()
