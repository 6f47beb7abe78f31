"""Committed golden fixtures (tests/golden/*.npz, made by
tests/golden/make_golden.py from the oracle).

CPU: the oracle still produces them (regression pin of the restatement), and
the product's generator and C++ host setup match them bitwise (matrix hash,
aggregates, P, coarse operators, coarsest inverse).
GPU: the HIP apply matches the stored z (1e-10) and the device PCG takes the
stored number of iterations with residuals within 1e-6.
"""
import glob
import hashlib
import os

import numpy as np
import pytest

import mamg_oracle as mo

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, 'golden', '*.npz')))


def load(p):
    return dict(np.load(p, allow_pickle=False))


def sha(indptr, indices, data):
    h = hashlib.sha256()
    for a in (np.asarray(indptr, np.int64), np.asarray(indices, np.int32), np.asarray(data, np.float64)):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def case(d):
    return int(d['dim']), int(d['n']), float(d['gamma'])


def test_fixtures_present():
    assert len(FIXTURES) == 6


@pytest.mark.parametrize('path', FIXTURES, ids=os.path.basename)
def test_oracle_reproduces_fixture(path):
    d = load(path)
    dim, n, g = case(d)
    s = mo.bidomain_system(dim, n, g)
    A = s['A'].tocsr()
    assert sha(A.indptr, A.indices, A.data) == str(d['A_sha256'])
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s['idofs'])
    assert len(h.levels) == int(d['nlevels'])
    for l, lv in enumerate(h.levels):
        if l > 0:
            assert np.array_equal(lv.A.indptr, d['A%d_indptr' % l])
            assert np.array_equal(lv.A.indices, d['A%d_indices' % l])
            assert np.array_equal(lv.A.data, d['A%d_data' % l])
        if lv.P is not None:
            assert np.array_equal(lv.agg, d['agg%d' % l])
            assert np.array_equal(lv.P.data, d['P%d_data' % l])
    r = mo.seeded_rhs(A.shape[0], 1234)
    z = h.apply(r)
    assert np.linalg.norm(z - d['z']) / np.linalg.norm(d['z']) < 1e-12
    cg = mo.pcg(A, h, r, 1e-8, 500)
    assert len(cg.residuals) == len(d['residuals'])
    assert np.allclose(cg.residuals, d['residuals'], rtol=1e-8, atol=0)


@pytest.mark.parametrize('path', FIXTURES, ids=os.path.basename)
def test_host_setup_matches_fixture(lib_built, path):
    import metric_amg_examples_amd as M
    d = load(path)
    dim, n, g = case(d)
    s = M.problems.bidomain(dim, n, g)
    assert sha(s.indptr, s.indices, s.data) == str(d['A_sha256'])
    H = M.HostHierarchy(s, idofs=s.idofs, num_functions=2)
    assert H.num_levels == int(d['nlevels'])
    for l in range(H.num_levels):
        lv = H.level(l, with_A=(l > 0))
        if l > 0:
            ip, ix, dv, _ = lv['A']
            assert np.array_equal(ip, d['A%d_indptr' % l])
            assert np.array_equal(ix, d['A%d_indices' % l])
            assert np.array_equal(dv, d['A%d_data' % l])
        if 'agg%d' % l in d:
            assert np.array_equal(lv['agg'], d['agg%d' % l])
            ip, ix, dv, _ = lv['P']
            assert np.array_equal(ip, d['P%d_indptr' % l])
            assert np.array_equal(ix, d['P%d_indices' % l])
            assert np.array_equal(dv, d['P%d_data' % l])
        else:
            assert np.array_equal(lv['Ainv'].reshape(d['Ainv'].shape), d['Ainv'])
    H.close()


@pytest.mark.gpu
@pytest.mark.parametrize('path', FIXTURES, ids=os.path.basename)
def test_gpu_apply_and_pcg_match_fixture(lib_built, path):
    import metric_amg_examples_amd as M
    d = load(path)
    dim, n, g = case(d)
    s = M.problems.bidomain(dim, n, g)
    B = M.MetricAMG(s.scipy(), s.W, idofs=s.idofs, num_functions=2)
    r = M.problems.seeded_rhs(s.N)
    z = B * r
    assert np.linalg.norm(z - d['z']) / np.linalg.norm(d['z']) < 1e-10
    solver = M.ConjGrad(s.scipy(), precond=B, tolerance=1e-8, maxiter=500)
    solver * r
    assert len(solver.residuals) == len(d['residuals'])
    assert np.allclose(solver.residuals, d['residuals'], rtol=1e-6, atol=0)
    B.close()
