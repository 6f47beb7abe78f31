"""CPU checks of the node-patch Schwarz restatement (mamg_oracle.Patches) and
of the C-ABI's parameter checks for SCHWARZ_PATCHES (no GPU needed).

* the distance-3 colouring is valid: two patch centres of one colour are at
  least 4 node hops apart, so no patch of a colour reads an x another writes;
* a colour-ordered sweep equals the same patches applied one at a time in
  that order (the parallel order is a multiplicative Schwarz order);
* the patch inverse is the inverse of the patch matrix;
* PCG iterations with the node patches stay within 1.5x of the reference
  algorithm restated on the CPU (oracle/ref_profile.py, src/amg_parameters.py:67-89).
"""
import numpy as np
import pytest
import scipy.sparse as sp

import mamg_oracle as mo


def _setup(dim, n, g, **kw):
    s = mo.bidomain_system(dim, n, g)
    h = mo.setup(s['A'], mo.Params(num_functions=2, Schwarz_type=mo.SCHWARZ_PATCHES, **kw), idofs=s['idofs'])
    return s, h


@pytest.mark.parametrize('dim,n', [(2, 16), (3, 6)])
def test_patch_colouring_distance3(dim, n):
    s, h = _setup(dim, n, 1e6)
    P = h.levels[0].patches
    G = mo.node_pattern(s['A'], 2)
    nv = G.shape[0]
    Gd = (G + sp.identity(nv, format='csr')).astype(bool).astype(np.int32)
    G3 = (Gd @ Gd @ Gd).tocsr()
    for c in range(P.ncolours):
        I = P.crows[c]
        sub = G3[I][:, I]
        assert sub.nnz == len(I)        # only the diagonal: centres > 3 hops apart
    assert sorted(np.concatenate(P.crows).tolist()) == list(range(nv))


def test_patch_sweep_is_sequential_schwarz():
    s, h = _setup(2, 12, 1e3)
    A = s['A'].tocsr()
    P = h.levels[0].patches
    b = mo.seeded_rhs(A.shape[0], 3)
    x0 = mo.seeded_rhs(A.shape[0], 4)
    x = P.sweep(A, x0.copy(), b, True)
    y = x0.copy()
    for c in range(P.ncolours):
        for I in P.crows[c]:
            d = P.dofs[I][P.dofs[I] >= 0]
            k = len(d)
            y[d] += P.Minv[I, :k, :k] @ (b[d] - A[d] @ y)
    assert np.linalg.norm(x - y) <= 1e-12 * np.linalg.norm(y)


def test_patch_inverse():
    s, h = _setup(3, 5, 1e6)
    A = s['A'].tocsr()
    P = h.levels[0].patches
    for I in (0, 17, 60):
        d = P.dofs[I][P.dofs[I] >= 0]
        k = len(d)
        Ap = A[d][:, d].toarray()
        assert np.linalg.norm(P.Minv[I, :k, :k] @ Ap - np.eye(k)) < 1e-8
        assert np.array_equal(P.Minv[I, :k, :k], P.Minv[I, :k, :k].T)


def test_patch_iterations_close_to_reference_algorithm():
    from ref_profile import RefHierarchy, RefParams
    s, h = _setup(3, 8, 1e6)
    A = s['A']
    b = mo.seeded_rhs(A.shape[0])
    its = mo.pcg(A, h, b, 1e-8, 500).niters
    ref = mo.pcg(A, RefHierarchy(A, s['idofs'], RefParams()), b, 1e-8, 500).niters
    assert its <= 1.5 * ref, (its, ref)


def test_patch_params_rejected_where_unsupported(lib_built):
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(2, 8, 1e2)
    A = s.scipy()
    with pytest.raises(M._lib.MamgError) as ei:       # scalar system
        M.HostHierarchy(A, idofs=s.idofs, num_functions=1, Schwarz_type=6)
    assert ei.value.code == -4 and 'PATCHES' in str(ei.value)
    with pytest.raises(M._lib.MamgError) as ei:       # no seed on some nodes
        M.HostHierarchy(A, idofs=s.idofs[: len(s.idofs) // 2], num_functions=2, Schwarz_type=6)
    assert ei.value.code == -4 and 'seed' in str(ei.value)
    H = M.HostHierarchy(A, idofs=s.idofs, num_functions=2, Schwarz_type=6)
    assert H.num_levels >= 2
    H.close()
