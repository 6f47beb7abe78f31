"""CPU checks of the seed-ring Schwarz restatement (mamg_oracle.Rings,
Schwarz_type RINGS: the reference's SCHWARZ_SYMMETRIC on the interface
seeds' overlapping Schwarz_maxlvl-rings, src/utils.py:60-86, as the EMI
drivers call it, src/emi_3d.py:133-139) -- no GPU needed.

* the greedy colouring is valid: no block of a colour has a member in the
  closed neighbourhood of another block of that colour, so a colour's blocks
  neither share a dof nor read an x another one writes;
* a colour-ordered sweep equals the same blocks applied one at a time in that
  order (the parallel order is a multiplicative Schwarz order);
* the rest's GS inverses leave covered dofs alone and invert the uncovered
  part of each node block;
* one level-0 step is symmetric, so the V/W cycle without coarse scaling is
  a symmetric operator; the EMI PCG is gamma-robust.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import mamg_oracle as mo

REF_DEFAULT = dict(AMG_type='UA', cycle_type='W', smoother='SGS', relaxation=1.2, coarse_scaling=1,
                   aggregation_type='HEM', strong_coupled=0.1, Schwarz_levels=1, Schwarz_mmsize=100,
                   Schwarz_maxlvl=2, Schwarz_type=3, num_functions=2)     # src/utils.py:60-82


def _emi(dim, n, g):
    import metric_amg_examples_amd as M
    return M.problems.emi(dim, n, g)


def _setup(s, **kw):
    p = mo.Params(**dict(REF_DEFAULT, **kw))
    return mo.setup(s.scipy(), p, idofs=s.idofs)


@pytest.mark.parametrize('dim,n', [(3, 8), (2, 32)])
def test_ring_colouring_valid(dim, n):
    s = _emi(dim, n, 1e6)
    A = s.scipy()
    h = _setup(s)
    R = h.levels[0].rings
    assert h.params.Schwarz_type == mo.SCHWARZ_RINGS
    assert len(R.blocks) == len(s.idofs)                  # one block per seed, every seed kept
    G = (abs(A) + sp.identity(A.shape[0])).tocsr()
    G.data[:] = 1.0
    for c in range(R.ncolours):
        ks = R.cblocks[c]
        touched = np.zeros(A.shape[0], int)
        for k in ks:
            t = np.unique(G[R.blocks[k]].indices)
            touched[t] += 1
        for k in ks:   # a member of k lies only in k's own closed neighbourhood
            assert touched[R.blocks[k]].max() == 1
    # greedy: each block of colour c > 0 conflicts with one of every smaller colour
    assert R.ncolours >= 2


def test_ring_sweep_is_sequential_schwarz():
    s = _emi(3, 8, 1e4)
    A = s.scipy().tocsr()
    h = _setup(s)
    R = h.levels[0].rings
    b = mo.seeded_rhs(A.shape[0], 3)
    x0 = mo.seeded_rhs(A.shape[0], 4)
    for fwd in (True, False):
        x = R.sweep(A, x0.copy(), b, fwd)
        y = x0.copy()
        order = range(R.ncolours) if fwd else range(R.ncolours - 1, -1, -1)
        for c in order:
            for k in R.cblocks[c]:
                d = R.blocks[k]
                y[d] += R.Minv[k] @ (b[d] - A[d] @ y)
        assert np.linalg.norm(x - y) <= 1e-12 * np.linalg.norm(y)


def test_ring_blocks_and_inverses():
    s = _emi(3, 8, 1e6)
    A = s.scipy().tocsr()
    h = _setup(s)
    R = h.levels[0].rings
    for k in (0, 7, len(R.blocks) - 1):
        d = R.blocks[k]
        assert s.idofs[k] in d and len(d) <= 100 and np.all(np.diff(d) > 0)
        Ak = A[d][:, d].toarray()
        assert np.allclose(R.Minv[k] @ Ak, np.eye(len(d)), atol=1e-9)


def test_rest_gs_inverse_masks_covered_dofs():
    s = _emi(3, 8, 1e6)
    A = s.scipy().tocsr()
    h = _setup(s)
    L = h.levels[0]
    nv = A.shape[0] // 2
    cov = L.rings.cov
    d = A.diagonal()
    for I in range(nv):
        D = L.Dn[I]
        c0, c1 = cov[I], cov[nv + I]
        if c0 and c1:
            assert not D.any()
        elif c0:
            assert D[0, 0] == 0 and D[0, 1] == 0 and D[1, 0] == 0 and D[1, 1] == 1.0 / d[nv + I]
        elif c1:
            assert D[1, 1] == 0 and D[0, 1] == 0 and D[1, 0] == 0 and D[0, 0] == 1.0 / d[I]
        else:
            B = A[[I, nv + I]][:, [I, nv + I]].toarray()
            assert np.allclose(D @ B, np.eye(2), atol=1e-12)


@pytest.mark.parametrize('cycle', ['V', 'W'])
def test_rings_cycle_symmetric(cycle):
    s = _emi(3, 8, 1e6)
    h = _setup(s, coarse_scaling=0, cycle_type=cycle)
    r1, r2 = mo.seeded_rhs(s.N, 1), mo.seeded_rhs(s.N, 2)
    a, c = r2 @ h.apply(r1), r1 @ h.apply(r2)
    assert abs(a - c) <= 1e-10 * abs(a)
    assert r1 @ h.apply(r1) > 0


def test_rings_emi_pcg_gamma_robust():
    """The reference's EMI preconditioner (default dict) on EMI 3-D n = 8:
    a handful of PCG iterations at every gamma (tolerance 1e-10 as
    src/emi_3d.py:143)."""
    its = []
    for g in (1.0, 1e4, 1e8):
        s = _emi(3, 8, g)
        h = _setup(s)
        its.append(mo.pcg(s.scipy(), h, mo.seeded_rhs(s.N), 1e-10, 500).niters)
    assert max(its) <= 20, its


@pytest.mark.parametrize('dim,n,g', [(3, 8, 1e6), (3, 16, 1e6), (3, 16, 1.0), (2, 32, 1e6)])
def test_colour_order_vs_seed_order(dim, n, g):
    """the GPU sweeps the seed-ring blocks colour by colour; the
    reference's SCHWARZ_SYMMETRIC (recalled: HAZmath is absent) sweeps them
    in seed order.  Same blocks and local solves, two multiplicative orders:
    the EMI PCG counts (tolerance 1e-10, src/emi_3d.py:143) differ by at most
    one iteration, and both cycles stay symmetric (DESIGN.md 2.12 records the
    counts)."""
    s = _emi(dim, n, g)
    A = s.scipy()
    b = mo.seeded_rhs(s.N)
    h = _setup(s)
    its_col = mo.pcg(A, h, b, 1e-10, 500).niters
    h.levels[0].rings.seed_order = True
    its_seed = mo.pcg(A, h, b, 1e-10, 500).niters
    print('EMI %dD n=%d gamma=%g: PCG its colour order %d, seed order %d, colours %d, blocks %d'
          % (dim, n, g, its_col, its_seed, h.levels[0].rings.ncolours, len(h.levels[0].rings.blocks)))
    assert abs(its_col - its_seed) <= 1, (its_col, its_seed)
    hs = _setup(s, coarse_scaling=0)
    hs.levels[0].rings.seed_order = True
    r1, r2 = mo.seeded_rhs(s.N, 1), mo.seeded_rhs(s.N, 2)
    a, c = r2 @ hs.apply(r1), r1 @ hs.apply(r2)
    assert abs(a - c) <= 1e-10 * abs(a)


def test_resolution_of_the_reference_names():
    """SCHWARZ_SYMMETRIC resolves by the seeds (mirrors setup.cpp
    resolve_params): 1-rings with a seed on every node -> node patches,
    anything sparser or wider -> seed rings, no seeds -> no Schwarz level."""
    p = mo.Params(**REF_DEFAULT)
    nv = 10
    every = np.arange(nv, 2 * nv)
    assert mo.resolve_params(p, every, 2 * nv).Schwarz_type == mo.SCHWARZ_RINGS      # 2-rings
    p1 = mo.Params(**dict(REF_DEFAULT, Schwarz_maxlvl=1))
    assert mo.resolve_params(p1, every, 2 * nv).Schwarz_type == mo.SCHWARZ_PATCHES
    assert mo.resolve_params(p1, every[::2], 2 * nv).Schwarz_type == mo.SCHWARZ_RINGS
    assert mo.resolve_params(p1, None, 2 * nv).Schwarz_levels == 0
