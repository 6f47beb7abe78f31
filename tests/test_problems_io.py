"""CPU checks of the EMI / 3D-1D generators, the .npy / .dat / solution.txt
file boundary and the seed-pair rule; no GPU.

Generators are pinned by exact finite-element identities (linear functions
are integrated exactly by P1), not by the reference (FEniCS is absent:
parity unpinned)."""
import os

import numpy as np
import pytest

import mamg_oracle as mo

HERE = os.path.dirname(os.path.abspath(__file__))


def _M():
    import metric_amg_examples_amd as M
    return M


@pytest.mark.parametrize('dim,n,N', [(3, 64, 278850), (2, 64, 4290), (3, 4, 150)])
def test_emi_sizes(dim, n, N):
    if n == 64 and dim == 3:
        # size formula only (assembly of the full config is exercised on the GPU box)
        nv = (n + 1) ** 2 * (n // 2 + 1)
        assert 2 * nv == N
        return
    s = _M().problems.emi(dim, n, 1e3)
    assert s.N == N and s.W[0] == s.W[1]


@pytest.mark.parametrize('dim,n', [(2, 8), (3, 4), (3, 8)])
def test_emi_structure_and_energy(dim, n):
    M = _M()
    g, k1, k2 = 1e4, 2.0, 3.0
    s = M.problems.emi(dim, n, g, k1, k2)
    A = s.scipy()
    assert abs(A - A.T).max() == 0.0
    nv = s.W[0]
    ng = (n + 1) ** (dim - 1)
    # coupling only between interface layers; total interface mass = |Gamma| = 1
    A01 = s.blocks[0][1].tocoo()
    assert A01.row.max() < ng and A01.col.max() < ng
    assert abs(A01.sum() + g) < 1e-9 * g
    # exact energy of u1 = 1 - x_d on Omega_1 (zero on its Dirichlet face), u2 = 0:
    #   k1 |Omega_1| + g |Gamma| (1/2)^2
    h = 1.0 / n
    layer = np.arange(nv) // ng
    u = np.concatenate([0.5 - layer * h, np.zeros(nv)])
    assert abs(u @ (A @ u) - (k1 * 0.5 + g * 0.25)) < 1e-9 * (k1 + g)
    # same for u2 = x_d on Omega_2: k2 |Omega_2| + g (1/2)^2
    v = np.concatenate([np.zeros(nv), 0.5 - layer * h])
    assert abs(v @ (A @ v) - (k2 * 0.5 + g * 0.25)) < 1e-9 * (k2 + g)
    # SPD (small)
    if s.N < 1500:
        assert np.linalg.eigvalsh(A.toarray()).min() > 0
    # interface dofs: u1 side (2-D) / both sides (3-D), as the reference drivers pass them
    assert len(s.idofs) == (ng if dim == 2 else 2 * ng)


def test_neuron_curve_is_made_of_mesh_edges():
    M = _M()
    for n in (8, 16, 32):
        pts, edges = M.problems.neuron_curve(n)
        d = pts[edges[:, 1]] - pts[edges[:, 0]]
        ok = [tuple(x) in {(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 1)} for x in d]
        assert all(ok)
        assert pts.min() >= 0 and pts.max() <= n
        assert len(edges) == len(pts) - 1            # a tree


@pytest.mark.parametrize('radius', [0.0, 0.2, 1.0, 2.5])
def test_emi_3d1d_system(radius):
    M = _M()
    s = M.problems.emi_3d1d(8, 1e2, radius)
    A = s.scipy()
    assert abs(A - A.T).max() < 1e-12 * abs(A).max()
    # A10 = -gc M1 Avg: rows of Avg sum to 1, so row sums of A10 = -gc * M1 row sums
    gc = s.info['gamma_c']
    A10 = s.blocks[1][0]
    rs = np.asarray(A10.sum(axis=1)).ravel()
    assert rs.max() < 0
    assert np.linalg.eigvalsh(A.toarray()).min() > 0
    assert np.array_equal(s.idofs, np.arange(s.W[0], s.N))
    assert abs(gc - 1e2 * 2 * np.pi * (radius if radius > 0 else 1.0)) < 1e-9 * gc


def test_npy_triplet_round_trip(tmp_path):
    M = _M()
    s = M.problems.emi_3d1d(6, 1e3, 0.5)
    A = s.scipy()
    b = M.problems.seeded_rhs(s.N)
    M.fileio.dump_system(A, b, s.W, str(tmp_path))
    raw = np.load(tmp_path / 'A.npy')
    assert raw.shape == (A.nnz, 3) and raw.dtype == np.float64
    A2, b2, idofs, idofs3d = M.fileio.load_system(str(tmp_path))
    assert (A2 != A).nnz == 0 and np.array_equal(b2, b)
    assert np.array_equal(idofs, np.arange(s.W[0], s.N)) and np.array_equal(idofs3d, np.arange(s.W[0]))
    M.fileio.write_solution(str(tmp_path / 'solution.txt'), b)
    assert np.array_equal(M.fileio.read_solution(str(tmp_path / 'solution.txt')), b)
    with open(tmp_path / 'solution.txt') as f:
        assert int(f.readline()) == s.N


def test_dat_reader_and_mapping():
    M = _M()
    d = M.fileio.read_dat(os.path.join(HERE, 'golden', 'solver_3d1d.dat'))
    assert d['AMG_type'] == 'SA' and d['AMG_coarse_dof'] == 300 and d['linear_itsolver_tol'] == 1e-6
    prm, solver, notes = M.fileio.dat_to_parameters(d)
    P = M.parameters
    assert prm['AMG_type'] == P.SA_AMG and prm['cycle_type'] == P.V_CYCLE
    assert prm['smoother'] == P.SMOOTHER_JACOBI_RHO and prm['aggregation_type'] == P.VMB   # as the file says
    # HAZmath's multiplicative Schwarz on the 1-D seeds' 2-rings -> the
    # additive overlapping Schwarz on the same blocks
    assert prm['Schwarz_type'] == P.SCHWARZ_ADDITIVE and prm['Schwarz_mmsize'] == 200
    assert prm['Schwarz_maxlvl'] == 2 and any('SCHWARZ_ADDITIVE' in n for n in notes)
    assert prm['coarse_dof'] == 300 and prm['max_levels'] == 30
    assert solver == dict(type=1, maxit=1000, tol=1e-6, stop_type=1, precond_type=16)
    assert len(notes) >= 3
    P.make_params(prm)                       # every mapped key is a valid parameter


def test_seed_pairs_form_node_blocks(lib_built):
    """Seeds on both sides of the EMI interface are reduced to the second
    field's seed at the C-ABI (capi.cpp Seeds): the level-0 smoother then
    holds the coupled pair {u1_I, u2_I}, exactly as with one-sided seeds."""
    M = _M()
    s = M.problems.emi(3, 8, 1e6)
    A = s.scipy()
    nv, ng = s.W[0], s.info['n_interface']
    both = M.HostHierarchy(A, idofs=np.r_[np.arange(ng), nv + np.arange(ng)], num_functions=2)
    one = M.HostHierarchy(A, idofs=nv + np.arange(ng), num_functions=2)
    a, b = both.level(0, with_A=False), one.level(0, with_A=False)
    for k in ('WB', 'P', 'R'):
        for u, v in zip(a[k][:3], b[k][:3]):
            assert np.array_equal(u, v), k
    # the oracle with one-sided seeds is gamma-robust on EMI (both-sided: not)
    r = mo.seeded_rhs(s.N)
    h = mo.setup(A, mo.Params(num_functions=2), idofs=nv + np.arange(ng))
    assert mo.pcg(A, h, r, 1e-10, 500, relativeconv=True).niters < 60


def test_reduction_operator():
    M = _M()
    R = M.precond.ReductionOperator([3, 2])
    x = R([np.arange(3.0), np.arange(2.0) + 10])
    assert np.array_equal(x, [0, 1, 2, 10, 11])
    y = R.T(x)
    assert np.array_equal(y[0], [0, 1, 2]) and np.array_equal(y[1], [10, 11])
