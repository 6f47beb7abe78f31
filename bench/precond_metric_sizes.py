#!/usr/bin/env python3
"""the bidomain drivers' `-precond metric` call (src/bidomain_3d.py:
163-165: the block form without parameters, i.e. the default dict of
src/utils.py:60-82 -- SCHWARZ_SYMMETRIC on every u2 dof's 2-ring, which runs
as SCHWARZ_RINGS) at the driver's mesh sizes: setup wall time, HBM held, the
seed-ring blocks / colours / host colouring time (print_level 1 line on
stderr), PCG iterations; the first size past the dense-block limit is refused.

    python bench/precond_metric_sizes.py [--max-n 128]
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
    ap.add_argument('--max-n', type=int, default=128)
    args = ap.parse_args()
    import numpy as np
    import torch
    import metric_amg_examples_amd as M
    from metric_amg_examples_amd.precond import get_hazmath_metric_precond
    torch.cuda.init()
    n = 8
    while n <= args.max_n:
        s = M.problems.bidomain(3, n, 1e6)
        idofs = np.arange(s.nv, 2 * s.nv, dtype=np.int32)          # src/bidomain_3d.py:163
        free0 = torch.cuda.mem_get_info()[0]
        t0 = time.time()
        row = {'n': n, 'N': s.N, 'seeds': int(idofs.size)}
        try:
            BB = get_hazmath_metric_precond(s, s.W, interface_dofs=idofs, print_level=1)
            torch.cuda.synchronize()
            row['setup_s'] = round(time.time() - t0, 3)
            row['hbm_held_GB'] = round((free0 - torch.cuda.mem_get_info()[0]) / 1e9, 3)
            Minv = BB.monolithic
            row['schwarz'] = Minv.effective_params['Schwarz_type']
            cg = M.ConjGrad(BB.Aop, precond=BB, tolerance=1e-8, maxiter=500)
            t1 = time.time()
            cg * M.problems.seeded_rhs(s.N)
            row['pcg_its'] = len(cg.residuals) - 1
            row['pcg_s'] = round(time.time() - t1, 3)
            Minv.close()
        except M._lib.MamgError as e:
            row['refused'] = str(e)
        print(json.dumps(row), flush=True)
        n *= 2


if __name__ == '__main__':
    main()
