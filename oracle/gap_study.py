"""Iteration-count gap between the reference's metric_mono algorithm
(ref_profile.py, HAZmath restated: UA + HEM + W-cycle + SGS + symmetric
multiplicative Schwarz + coarse scaling) and the GPU profile mi355x_sa_v
(mamg_oracle.py: nodal SA + V-cycle + block Jacobi), both under cbc.block
ConjGrad (tolerance 1e-8 absolute, maxiter 500; src/bidomain_3d.py:149).
Test infrastructure: writes oracle/gap_study.json.

    python oracle/gap_study.py [--quick]
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import mamg_oracle as mo          # noqa: E402
from ref_profile import RefHierarchy, RefParams   # noqa: E402


def run(cases, gammas):
    rows = []
    for dim, n in cases:
        for g in gammas:
            s = mo.bidomain_system(dim, n, g)
            A = s['A']
            b = mo.seeded_rhs(A.shape[0])
            t0 = time.time()
            href = RefHierarchy(A, s['idofs'], RefParams())
            cref = mo.pcg(A, href, b, 1e-8, 500)
            t1 = time.time()
            hgpu = mo.setup(A, mo.Params(num_functions=2), idofs=s['idofs'])
            cgpu = mo.pcg(A, hgpu, b, 1e-8, 500)
            row = dict(dim=dim, n=n, N=int(A.shape[0]), gamma=g, ref_metric_mono=cref.niters,
                       ref_levels=len(href.levels), mi355x_sa_v=cgpu.niters, gpu_levels=len(hgpu.levels),
                       ref_seconds=round(t1 - t0, 2))
            rows.append(row)
            print(row, flush=True)
    return rows


if __name__ == '__main__':
    quick = '--quick' in sys.argv
    cases = [(2, 32), (3, 8)] if quick else [(2, 32), (2, 64), (3, 8), (3, 16)]
    gammas = [1.0, 1e4, 1e8] if quick else [1.0, 1e2, 1e4, 1e6, 1e8, 1e10]
    rows = run(cases, gammas)
    if not quick:
        with open(os.path.join(HERE, 'gap_study.json'), 'w') as f:
            json.dump(rows, f, indent=1)
