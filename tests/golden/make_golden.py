#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU
oracle (oracle/mamg_oracle.py), as SURVEY.md section 8(c) plans:

    python tests/golden/make_golden.py

Cases: 2-D bidomain n = 32 and 64 and 3-D n = 8, gamma in {1, 1e6}, profile
mi355x_sa_v with nodal aggregation (num_functions = 2, seeds = u2 dofs).
Each fixture holds
  * a SHA-256 of the generated level-0 CSR (the matrix itself is regenerated),
  * per level: aggregates, P (CSR triplet), coarse A (CSR triplet),
  * the coarsest dense inverse,
  * one apply z = B r for r = seeded_rhs(N, 1234),
  * the PCG residual history (tolerance 1e-8 absolute, maxiter 500, b = r).
These are the oracle's own outputs: they freeze the restatement (a change to
the oracle, the C++ setup or the HIP apply shows up against stored data),
they do not pin it to HAZmath (parity unpinned).
Loaded with numpy.load (allow_pickle=False).
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', '..', 'oracle'))
import mamg_oracle as mo  # noqa: E402

CASES = [(2, 32, 1.0), (2, 32, 1e6), (2, 64, 1.0), (2, 64, 1e6), (3, 8, 1.0), (3, 8, 1e6)]


def name(dim, n, g):
    return 'bidomain%dd_n%d_g%g.npz' % (dim, n, g)


def csr_sha(A):
    h = hashlib.sha256()
    for a in (A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data.astype(np.float64)):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def make(dim, n, g):
    s = mo.bidomain_system(dim, n, g)
    A = s['A'].tocsr()
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s['idofs'])
    r = mo.seeded_rhs(A.shape[0], 1234)
    z = h.apply(r)
    cg = mo.pcg(A, h, r, 1e-8, 500)
    out = {'dim': np.int64(dim), 'n': np.int64(n), 'gamma': np.float64(g),
           'N': np.int64(A.shape[0]), 'nnz': np.int64(A.nnz),
           'A_sha256': np.array(csr_sha(A)), 'nlevels': np.int64(len(h.levels)),
           'z': z, 'residuals': np.asarray(cg.residuals, dtype=np.float64)}
    for l, lv in enumerate(h.levels):
        if l > 0:
            out['A%d_indptr' % l] = lv.A.indptr.astype(np.int64)
            out['A%d_indices' % l] = lv.A.indices.astype(np.int32)
            out['A%d_data' % l] = lv.A.data
        if lv.P is not None:
            out['agg%d' % l] = lv.agg.astype(np.int64)
            out['P%d_indptr' % l] = lv.P.indptr.astype(np.int64)
            out['P%d_indices' % l] = lv.P.indices.astype(np.int32)
            out['P%d_data' % l] = lv.P.data
        if lv.Ainv is not None:
            out['Ainv'] = lv.Ainv
    return out


def main():
    for dim, n, g in CASES:
        d = make(dim, n, g)
        p = os.path.join(HERE, name(dim, n, g))
        np.savez_compressed(p, **d)
        print('%s: N=%d levels=%d niters=%d size=%d B' % (os.path.basename(p), d['N'], d['nlevels'],
                                                         len(d['residuals']) - 1, os.path.getsize(p)))


if __name__ == '__main__':
    main()
