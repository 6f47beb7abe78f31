"""Manufactured solutions of the bidomain drivers (src/bidomain_2d.py:7-99,
:239-256; src/bidomain_3d.py:7-49): csrc/mms.cpp against the numpy
restatement (oracle/mms_ref.py), and the discretisation's H1 convergence rate
(the reference's own sanity pin: rate ~1 for P1) with direct solves."""
import numpy as np
import pytest
import scipy.sparse.linalg as spla

import mms_ref


@pytest.mark.parametrize('dim,n,gamma', [(2, 8, 5.0), (2, 16, 1e6), (3, 4, 1.0), (3, 8, 1e4)])
def test_mms_cpp_matches_numpy_restatement(lib_built, dim, n, gamma):
    from metric_amg_examples_amd import problems
    ref = mms_ref.BidomainMMS(dim, n, gamma, 2.0, 3.0)
    b = problems.bidomain_mms_rhs(dim, n, gamma, 2.0, 3.0)
    bo = ref.rhs()
    assert np.abs(b - bo).max() <= 1e-13 * np.abs(bo).max()
    # the lifting uses the generator's own element matrices: the eliminated
    # full matrix of the restatement is the generator's matrix
    s = problems.bidomain(dim, n, gamma)
    D = ref.dirichlet_nodes()
    Af = problems._eliminate(ref.full_matrix(), np.concatenate([D, ref.nv + D]))
    assert abs(s.scipy() - Af).max() <= 1e-12 * abs(Af).max()
    x = spla.spsolve(s.scipy().tocsc(), b)
    e = problems.bidomain_mms_errors(dim, n, x, gamma)
    eo = ref.h1_errors(x)
    assert np.allclose(e, eo, rtol=1e-12, atol=0)


@pytest.mark.parametrize('dim,ns,gamma,lo', [(2, (16, 32, 64), 1.0, 0.98), (2, (16, 32, 64), 1e6, 0.98),
                                              (3, (8, 16, 24), 5.0, 0.9)])
def test_mms_h1_rate_is_one(lib_built, dim, ns, gamma, lo):
    from metric_amg_examples_amd import problems
    errs, hs = [], []
    for n in ns:
        s = problems.bidomain(dim, n, gamma)
        x = spla.spsolve(s.scipy().tocsc(), problems.bidomain_mms_rhs(dim, n, gamma))
        errs.append(problems.bidomain_mms_errors(dim, n, x, gamma))
        hs.append(np.sqrt(dim) / n)
    errs = np.array(errs)
    rates = np.log(errs[1:] / errs[:-1]) / np.log(np.array(hs[1:]) / np.array(hs[:-1]))[:, None]
    assert np.all(rates[-1] > lo) and np.all(rates[-1] < 1.1), rates


def test_mms_rejects_bad_arguments(lib_built):
    from metric_amg_examples_amd import problems, _lib
    with pytest.raises(_lib.MamgError):
        problems.bidomain_mms_rhs(4, 8, 1.0)
    with pytest.raises(ValueError):
        problems.bidomain_mms_errors(2, 8, np.zeros(5), 1.0)


@pytest.mark.parametrize('dim,ns,gamma,lo', [(2, (16, 32, 64), 1.0, 0.98), (2, (16, 32, 64), 1e6, 0.98),
                                              (3, (4, 8, 16), 5.0, 0.9)])
def test_emi_mms_h1_rate_is_one(lib_built, dim, ns, gamma, lo):
    """EMI manufactured solution (src/emi_2d.py:8-128: interface terms g_r, g_n,
    full flux on the sides, Dirichlet on the outer faces): H1 rate ~1 with
    direct solves of problems.emi -- a sign or normal error would stall it."""
    from metric_amg_examples_amd import mms, problems
    errs = []
    for n in ns:
        s = problems.emi(dim, n, gamma)
        b = np.concatenate(mms.emi_mms_rhs(dim, n, gamma))
        x = spla.spsolve(s.scipy().tocsc(), b)
        errs.append(mms.emi_mms_errors(dim, n, x, gamma))
    errs = np.array(errs)
    rates = np.log(errs[1:] / errs[:-1]) / np.log(0.5)
    assert np.all(rates[-1] > lo) and np.all(rates[-1] < 1.1), rates
