#!/usr/bin/env python3
"""GPU vs host setup time for the hierarchies without 2x2 node-block
smoothers (csrc/gsetup.hip generic path): the 3D-1D system (scalar, additive
2-rings), EMI with the reference's overlapping 2-rings, scalar AMG on the
bidomain matrix.  Each line: N, levels, host setup s, GPU setup s (MetricAMG
wall incl. A0 upload and layout), GPU setup phases, and whether the two
handles' applies are bitwise equal.

    python bench/setup_generic.py [--big]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--big', action='store_true')
    args = ap.parse_args()
    import metric_amg_examples_amd as M
    P = M.parameters
    cases = []
    s = M.problems.emi_3d1d(48, 1e4, 1.0)
    cases.append(('emi_3d1d n=48 radius 1', s.scipy(), s.W, s.idofs, dict(parameters=P.parameters_metric_3d1d)))
    s = M.problems.emi(3, 32, 1e6)
    cases.append(('emi_3d n=32 rings2 additive', s.tocsr(), s.W, s.idofs,
                  dict(num_functions=2, Schwarz_type=P.SCHWARZ_ADDITIVE, Schwarz_maxlvl=2)))
    cases.append(('emi_3d n=32 seed blocks', s.tocsr(), s.W, s.idofs, dict(num_functions=2)))
    nb = 128 if args.big else 64
    s = M.problems.bidomain(3, nb, 1e6)
    cases.append(('bidomain_3d n=%d scalar AMG' % nb, s.scipy(), None, None, dict(num_functions=1)))
    w = M.problems.bidomain(2, 16, 1.0)          # HIP context and code objects loaded before timing
    M.MetricAMG(w.scipy(), num_functions=1, setup='gpu').close()
    for name, A, W, idofs, kw in cases:
        out = {'case': name, 'N': A.shape[0], 'nnz': int(A.nnz)}
        for path in ('host', 'gpu'):
            t = time.perf_counter()
            B = M.MetricAMG(A, W, idofs=idofs, setup=path, **kw)
            out[path + '_s'] = round(time.perf_counter() - t, 3)
            if path == 'gpu':
                out['gpu_phases_ms'] = B.setup_timings
                Bg = B
            else:
                Bh = B
        out['levels'] = Bg.num_levels
        out['layout'] = Bg.layout
        r = M.problems.seeded_rhs(A.shape[0])
        out['apply_bitwise'] = bool(np.array_equal(Bg * r, Bh * r))
        out['speedup'] = round(out['host_s'] / out['gpu_s'], 2)
        print(json.dumps(out), flush=True)
        Bg.close()
        Bh.close()


if __name__ == '__main__':
    main()
