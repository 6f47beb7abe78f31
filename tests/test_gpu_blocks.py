"""GPU: the block-form preconditioner R^T Minv R on the EMI systems, the
file-based 3D-1D solve and the drivers, against the
CPU oracle on the same matrices.

Parity: the hierarchy is bitwise the oracle's (tests/test_host_setup.py,
tests/test_gpu_setup.py), so a PCG through the GPU preconditioner takes the
oracle's iteration count; residual histories agree to 1e-6 relative.
"""
import os

import numpy as np
import pytest

import mamg_oracle as mo

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _M():
    import metric_amg_examples_amd as M
    return M


def one_sided(s):
    """the seed-pair rule (capi.cpp Seeds) applied to the driver's idofs"""
    nv = s.W[0]
    seeds = set(int(i) for i in s.idofs)
    return np.array(sorted(i for i in seeds if not (i < nv and i + nv in seeds)), np.int32)


@pytest.mark.parametrize('dim,n,g', [(2, 64, 1e6), (3, 16, 1e6), (3, 16, 1.0), (3, 8, 1e10)])
def test_emi_block_form_pcg_matches_oracle(lib_built, dim, n, g):
    M = _M()
    s = M.problems.emi(dim, n, g)
    # the GPU profile (explicit; parameters=None is the reference's default
    # dict, tests/test_gpu_rings.py)
    BB = M.precond.get_hazmath_metric_precond(s.blocks, s.W, parameters=M.parameters.parameters_metric_mi355x,
                                              interface_dofs=s.idofs, num_functions=2)
    # interface seeds recruit their own side's interior neighbours: blocks are
    # not node-aligned, so the GPU setup builds a general block smoother and
    # the handle runs the CSR layout
    assert BB.monolithic.setup_path == 'gpu'
    assert BB.monolithic.layout == 'csr'
    b = [M.problems.seeded_rhs(s.W[0], 1234), M.problems.seeded_rhs(s.W[1], 4321)]
    # block apply == monolithic apply
    z = BB * b
    zm = BB.monolithic * np.concatenate(b)
    assert np.array_equal(np.concatenate(z), zm)
    solver = M.ConjGrad(s, precond=BB, tolerance=1e-10, maxiter=500)     # src/emi_3d.py:143
    x = solver * b
    A = s.scipy()
    h = mo.setup(A, mo.Params(num_functions=2), idofs=one_sided(s))
    ref = mo.pcg(A, h, np.concatenate(b), 1e-10, 500)
    assert len(solver.residuals) == len(ref.residuals)
    assert np.allclose(solver.residuals, ref.residuals, rtol=1e-6, atol=0)
    assert len(solver.residuals) < 80                                  # gamma-robust
    assert isinstance(x, list) and len(x[0]) == s.W[0]


@pytest.mark.parametrize('dim,n,g', [(3, 16, 1e6), (2, 64, 1e6), (3, 8, 1e10)])
def test_emi_reference_rings_gpu_setup(lib_built, dim, n, g):
    """The reference's EMI smoother blocks: the interface seeds' overlapping
    2-rings (get_hazmath_metric_precond_mono's Schwarz_maxlvl 2,
    /root/reference/src/utils.py:60-86), smoothed additively
    (SCHWARZ_ADDITIVE), built by the GPU setup: PCG history of the oracle."""
    M = _M()
    P = M.parameters
    s = M.problems.emi(dim, n, g)
    A = s.tocsr()
    kw = dict(num_functions=2, Schwarz_type=P.SCHWARZ_ADDITIVE, Schwarz_maxlvl=2)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, **kw)
    assert B.setup_path == 'gpu' and B.layout == 'csr'
    b = M.problems.seeded_rhs(s.N, 1234)
    solver = M.ConjGrad(A, precond=B, tolerance=1e-10, maxiter=500)
    solver * b
    h = mo.setup(A, mo.Params(num_functions=2, Schwarz_type=5, Schwarz_maxlvl=2), idofs=one_sided(s))
    ref = mo.pcg(A, h, b, 1e-10, 500)
    if g < 1e8:
        assert len(solver.residuals) == len(ref.residuals)
        assert np.allclose(solver.residuals, ref.residuals, rtol=1e-6, atol=0)
    else:
        assert abs(len(solver.residuals) - len(ref.residuals)) <= 1
    assert len(solver.residuals) < 80


@pytest.mark.parametrize('dim,n,g,kw', [(3, 16, 1e6, {}), (3, 32, 1e6, dict(smoother=12)),
                                        (2, 128, 1e6, dict(smoother=12)), (3, 8, 1e10, {})])
def test_emi_node_aligned_seeds_gpu_setup(lib_built, dim, n, g, kw):
    """Schwarz_maxlvl 0: the interface seeds' blocks are their nodes (u0_I,
    u1_I mirror pairs), so every level is node-aligned: GPU setup, BSR2 layout
    (the multi-GPU path's format), and the PCG history of the oracle."""
    M = _M()
    s = M.problems.emi(dim, n, g)
    A = s.tocsr()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, Schwarz_maxlvl=0, **kw)
    assert B.setup_path == 'gpu' and B.layout == 'bsr2'
    b = M.problems.seeded_rhs(s.N, 1234)
    solver = M.ConjGrad(A, precond=B, tolerance=1e-10, maxiter=500)     # src/emi_3d.py:143
    assert solver._device_ok()                                         # device-resident PCG
    solver * b
    okw = dict(smoother='POLY') if kw.get('smoother') == 12 else {}
    h = mo.setup(A, mo.Params(num_functions=2, Schwarz_maxlvl=0, **okw), idofs=s.idofs)
    ref = mo.pcg(A, h, b, 1e-10, 500)
    if g < 1e8:
        assert len(solver.residuals) == len(ref.residuals)
        assert np.allclose(solver.residuals, ref.residuals, rtol=1e-6, atol=0)
    else:   # conditioning (entries span gamma) amplifies summation order: the late
        # residuals, near the 1e-10 absolute stop, drift; the count may move by one
        assert abs(len(solver.residuals) - len(ref.residuals)) <= 1
        assert np.allclose(solver.residuals[:4], ref.residuals[:4], rtol=1e-6, atol=0)
    assert len(solver.residuals) < 80


def _oracle_pcg_relres(A, h, b, tol, maxit):
    """PCG stopped on ||r||/||b|| (HAZmath linear_stop_type 1)."""
    x = np.zeros_like(b)
    r = b.copy()
    z = h.apply(r)
    d = z.copy()
    rz = r @ z
    bn = np.linalg.norm(b)
    it = 0
    while np.linalg.norm(r) > tol * bn and it < maxit:
        q = A @ d
        al = rz / (d @ q)
        x += al * d
        r -= al * q
        z = h.apply(r)
        rz2 = r @ z
        d = z + (rz2 / rz) * d
        rz = rz2
        it += 1
    return x, it


@pytest.mark.parametrize('radius,g', [(0.0, 1e2), (0.0, 1e8), (1.0, 1e4), (2.5, 1e2), (1.0, 1e6), (2.5, 1e8)])
def test_file_based_3d1d_solve(lib_built, tmp_path, radius, g):
    """emi_3d1d -dump 1 -> run_solver_3d1d (haznics.fenics_metric_solver_xd_1d
    restated) -> solution.txt; iteration count = the oracle's with the same
    parameters and stopping rule."""
    M = _M()
    s = M.problems.emi_3d1d(16, g, radius)
    A = s.scipy()
    b = M.problems.seeded_rhs(s.N)
    mdir, odir = tmp_path / 'mat', tmp_path / 'out'
    M.fileio.dump_system(A, b, s.W, str(mdir))
    from metric_amg_examples_amd import drivers
    dat = os.path.join(HERE, 'golden', 'solver_3d1d.dat')
    niters = drivers.fenics_metric_solver_xd_1d(dat, str(mdir) + '/', str(odir) + '/', quiet=True)
    x = M.fileio.read_solution(str(odir / 'solution.txt'))
    assert np.linalg.norm(b - A @ x) <= 1e-6 * np.linalg.norm(b) * (1 + 1e-9)
    # the file's Schwarz (maxlvl 2, mmsize 200) -> additive overlapping rings
    prm = mo.Params(coarse_dof=300, max_levels=30, Schwarz_mmsize=200, Schwarz_type=5, Schwarz_maxlvl=2,
                    aggregation_type='VMB')      # AMG_aggregation_type 1, as the file says
    h = mo.setup(A, prm, idofs=s.idofs)
    xo, it = _oracle_pcg_relres(A, h, b, 1e-6, 1000)
    assert niters == it
    assert niters < 120            # gamma-robust with the averaged coupling too
    assert np.linalg.norm(x - xo) <= 1e-6 * np.linalg.norm(xo)


def test_drivers_write_reference_iters_schema(lib_built, tmp_path):
    from metric_amg_examples_amd import drivers
    rows = drivers.bidomain(['-nrefs', '2', '-gamma', '1e6', '-precond', 'metric_mono',
                             '-results', str(tmp_path)], 2)
    assert len(rows) == 2 and rows[1][0] > rows[0][0]
    f = [p for p in os.listdir(tmp_path / 'bidomain_2d') if p.startswith('iters_precondmetric_mono')]
    lines = open(tmp_path / 'bidomain_2d' / f[0]).read().split('\n')
    assert lines[0] == 'ndofs niters cond timeKSP r h' and len(lines[1].split()) == 6
    # manufactured solution (the default right-hand side): the reference's
    # error table with H1 rate ~1, errors equal to the direct solve's
    f = [p for p in os.listdir(tmp_path / 'bidomain_2d') if p.startswith('error_precondmetric_mono')]
    lines = open(tmp_path / 'bidomain_2d' / f[0]).read().strip().split('\n')
    assert lines[0] == 'ndofs h |eu1|_1 r|eu1|_1 |eu2|_1 r|eu2|_1' and len(lines) == 3
    last = [float(v) for v in lines[2].split()]
    assert 0.97 < last[3] < 1.03 and 0.97 < last[5] < 1.03
    import scipy.sparse.linalg as spla
    from metric_amg_examples_amd import problems
    s = problems.bidomain(2, 64, 1e6)
    xd = spla.spsolve(s.scipy().tocsc(), problems.bidomain_mms_rhs(2, 64, 1e6))
    ed = problems.bidomain_mms_errors(2, 64, xd, 1e6)
    assert np.allclose([last[2], last[4]], ed, rtol=1e-6, atol=0)
    # -precond metric_hazmath: the whole solve in the library (solve_haznics), the same
    # preconditioner and CG as metric_mono here, so the same iteration count
    hz = drivers.bidomain(['-nrefs', '1', '-gamma', '1e6', '-precond', 'metric_hazmath',
                           '-results', str(tmp_path)], 2)
    assert hz[0][1] == rows[0][1] and hz[0][2] == -1
    rows = drivers.emi(['-nrefs', '1', '-gamma', '1e4', '-results', str(tmp_path)], 3)
    assert rows[0][1] < 30          # the reference's default dict: seed-ring Schwarz
    rows_g = drivers.emi(['-nrefs', '1', '-gamma', '1e4', '-profile', 'mi355x', '-results', str(tmp_path)], 3)
    assert rows_g[0][1] < 80
    rows = drivers.bidomain(['-nrefs', '1', '-gamma', '1e2', '-precond', 'metric',
                             '-results', str(tmp_path)], 3)
    assert rows[0][1] < 80
