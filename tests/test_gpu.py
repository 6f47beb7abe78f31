"""GPU parity: the HIP apply path (through the C-ABI) against the CPU oracle.

Tolerances (fp64): one preconditioner application z = B r agrees with the
oracle's to ||dz|| / ||z|| <= 1e-10 (the setup is bitwise identical; only
summation order inside the GPU SpMVs differs).  PCG: iteration count equal to
the oracle's, every residual within 1e-6 relative.  At full benchmark sizes
the checks are size-independent properties (symmetry, linearity, determinism
of graph replays, <Br, r> > 0).
"""
import numpy as np
import pytest

import mamg_oracle as mo
from conftest import set_opt

pytestmark = pytest.mark.gpu

APPLY_TOL = 1e-10


def _mamg():
    import metric_amg_examples_amd as M
    return M


def to_c(kw):
    c = dict(kw)
    if 'AMG_type' in c:
        c['AMG_type'] = {'SA': 2, 'UA': 1}[c['AMG_type']]
    if 'cycle_type' in c:
        c['cycle_type'] = {'V': 1, 'W': 2}[c['cycle_type']]
    if 'smoother' in c:
        c['smoother'] = {'JACOBI': 1, 'L1DIAG': 2, 'JACOBI_RHO': 3, 'GS': 10, 'SGS': 11,
                         'POLY': 12}[c['smoother']]
    return c


def rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


APPLY_CASES = [
    (2, 32, 1.0, dict(num_functions=2)),
    (2, 64, 1e6, dict(num_functions=2)),
    (3, 8, 1e6, dict(num_functions=2)),
    (3, 16, 1e4, dict(num_functions=2)),
    (3, 16, 1e10, dict(num_functions=2)),
    (3, 16, 1.0, dict()),
    (2, 32, 1e3, dict(AMG_type='UA', cycle_type='W')),
    (3, 16, 1e2, dict(num_functions=2, cycle_type='W')),
    (2, 32, 1e3, dict(num_functions=2, presmooth_iter=2, postsmooth_iter=3, maxit=2)),
    (2, 32, 1e3, dict(num_functions=2, node_block_smoother=0, sa_block_diag=0)),
    (3, 16, 1e6, dict(num_functions=2, post_fusion=0)),
    (2, 32, 1e3, dict(num_functions=2, post_fusion=0, cycle_type='W')),
    # SMOOTHER_POLY (Chebyshev steps w_k W): BSR2 with K built for w_m W, the
    # [P | AP] and unfused posts, sweeps > 1, W-cycle, and the CSR layout
    (3, 16, 1e6, dict(num_functions=2, smoother='POLY')),
    (2, 64, 1e6, dict(num_functions=2, smoother='POLY', poly_degree=3)),
    (3, 8, 1e2, dict(num_functions=2, smoother='POLY', post_fusion=0)),
    (2, 32, 1e3, dict(num_functions=2, smoother='POLY', presmooth_iter=2, postsmooth_iter=2,
                      cycle_type='W', maxit=2)),
    (3, 16, 1.0, dict(smoother='POLY')),
    (2, 32, 1e3, dict(num_functions=2, smoother='POLY', node_block_smoother=0, sa_block_diag=0,
                      poly_ratio=8.0)),
]
DEVICE_ONLY = ('post_fusion',)       # schedule knobs: same cycle, no oracle counterpart


def oracle_kw(kw):
    return {k: v for k, v in kw.items() if k not in DEVICE_ONLY}


@pytest.mark.parametrize('dim,n,g,kw', APPLY_CASES)
def test_apply_matches_oracle(lib_built, dim, n, g, kw):
    import torch
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    # num_functions explicit: MetricAMG would take 2 from the two equal blocks of W
    B = M.MetricAMG(A, s.W, idofs=s.idofs, **to_c(dict(dict(num_functions=1), **kw)))
    h = mo.setup(A, mo.Params(**oracle_kw(kw)), idofs=s.idofs)
    assert B.num_levels == len(h.levels)
    # gamma >= 1e8 makes A_l badly conditioned (entries span ~gamma); the
    # summation-order difference is then amplified: 1e-8 there
    tol = APPLY_TOL if g < 1e8 else 1e-8
    for seed in (1234, 7):
        r = mo.seeded_rhs(s.N, seed)
        zo = h.apply(r)
        z = B * r                                   # host pointers
        assert rel(z, zo) < tol
        zt = B.matvec(torch.as_tensor(r).cuda())    # device pointers, graph
        torch.cuda.synchronize()
        assert rel(zt.cpu().numpy(), zo) < tol


@pytest.mark.parametrize('dim,n,g,kw', [(2, 64, 1.0, {}), (3, 16, 1e6, {}), (3, 16, 1e10, {}), (2, 128, 1e4, {}),
                                        (3, 16, 1e6, dict(smoother='POLY')),
                                        (3, 32, 1e6, dict(smoother='POLY')),
                                        (2, 128, 1e4, dict(smoother='POLY'))])
def test_pcg_iterations_match_oracle(lib_built, dim, n, g, kw):
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    b = mo.seeded_rhs(s.N)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **to_c(kw))
    solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)   # device PCG
    x = solver * b
    h = mo.setup(A, mo.Params(num_functions=2, **kw), idofs=s.idofs)
    ref = mo.pcg(A, h, b, 1e-8, 500)
    assert len(solver.residuals) == len(ref.residuals)
    assert np.allclose(solver.residuals, ref.residuals, rtol=1e-6, atol=0)
    assert rel(x, ref.x) < 1e-6
    e1, e2 = solver.eigenvalue_estimates(), ref.eigenvalue_estimates()
    assert abs(e1[-1] / e1[0] - e2[-1] / e2[0]) < 1e-4 * (e2[-1] / e2[0])
    # host-loop ConjGrad (cbc.block structure, B*r through the C-ABI) agrees too
    host = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500, device=False)
    xh = host * b
    assert len(host.residuals) == len(ref.residuals)
    assert rel(xh, ref.x) < 1e-6


def test_callback_and_relativeconv(lib_built):
    M = _mamg()
    s = M.problems.bidomain(2, 32, 1e2)
    A = s.scipy()
    b = mo.seeded_rhs(s.N)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    seen = []
    solver = M.ConjGrad(A, precond=B, tolerance=1e-6, maxiter=200, relativeconv=True,
                        callback=lambda k, x, r: seen.append(k))
    solver * b
    assert seen == list(range(len(solver.residuals) - 1))
    assert solver.residuals[-1] <= 1e-6 * solver.residuals[0]


def test_spmv_matches_scipy(lib_built):
    import torch
    M = _mamg()
    s = M.problems.bidomain(3, 16, 1e3)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    x = np.random.default_rng(3).standard_normal(s.N)
    y = torch.empty(s.N, dtype=torch.float64, device='cuda')
    B.spmv_device(torch.as_tensor(x).cuda(), y)
    torch.cuda.synchronize()
    assert rel(y.cpu().numpy(), A @ x) < 1e-14


@pytest.mark.parametrize('lanes', [2, 4, 8, 16, 32, 64])
def test_lane_widths_agree(lib_built, lanes):
    M = _mamg()
    s = M.problems.bidomain(3, 8, 1e4)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, spmv_lanes=lanes)
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    assert rel(B * r, h.apply(r)) < APPLY_TOL


@pytest.mark.parametrize('dim,n,g,kw', [(3, 16, 1e4, dict(cycle_type='W')), (2, 64, 1.0, dict(maxit=2)),
                                        (3, 8, 1e6, dict(presmooth_iter=2, postsmooth_iter=2))])
def test_bsr2_and_csr_layouts_agree(lib_built, dim, n, g, kw):
    """The nodal hierarchy runs in the BSR2 layout; forcing the CSR layout
    (point smoothers are not block-fusable) must not change the cycle beyond
    summation order when the math is the same -- compare both to the oracle."""
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **to_c(kw))
    assert B.layout == 'bsr2'
    h = mo.setup(A, mo.Params(num_functions=2, **kw), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    assert rel(B * r, zo) < APPLY_TOL
    # same hierarchy uploaded in the CSR layout (host hierarchy -> mamg_upload)
    # point smoothers everywhere (no seeds, no node blocks) -> CSR layout
    Bc = M.MetricAMG(A, s.W, idofs=None, num_functions=2, node_block_smoother=0, **to_c(kw))
    assert Bc.layout == 'csr'
    hc = mo.setup(A, mo.Params(num_functions=2, node_block_smoother=0, **kw), idofs=None)
    assert rel(Bc * r, hc.apply(r)) < APPLY_TOL


@pytest.mark.parametrize('dim,n,g,kw', [(3, 16, 1e6, dict()), (3, 16, 1e4, dict(cycle_type='W')),
                                        (2, 64, 1.0, dict(maxit=2, postsmooth_iter=3)),
                                        (3, 8, 1e2, dict(presmooth_iter=2, postsmooth_iter=2))])
def test_post_fusion_equals_unfused(lib_built, dim, n, g, kw):
    """z = x1 + P e + W (r1 - (AP) e) (one pass over [P | AP]) is the same
    cycle as prolongation followed by a block-Jacobi sweep: fused and unfused
    schedules agree to summation order."""
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    Bf = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **to_c(kw))
    Bu = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, post_fusion=0, **to_c(kw))
    assert Bf.layout == Bu.layout == 'bsr2'
    for seed in (1234, 99):
        r = mo.seeded_rhs(s.N, seed)
        assert rel(Bf * r, Bu * r) < 1e-12


@pytest.mark.parametrize('sell', ['0', '1'])
def test_post_operator_k_equals_merged(lib_built, monkeypatch, sell):
    """K = P - W (A P) stored as one operator (z = x1 + W r1 + K e, default)
    and the merged [P | AP] window (z = x1 + P e + W (r1 - AP e)) are the
    same cycle up to summation order."""
    M = _mamg()
    set_opt('MAMG_SELL_MIN_ROWS', '1' if sell == '1' else str(1 << 20))
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    zs, fmts = [], []
    for k in ('1', '0'):
        set_opt('MAMG_POST_K', k)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        fmts.append(B.level_format(0))
        zs.append(B * mo.seeded_rhs(s.N))
        B.close()
    assert fmts[0]['post_k'] and not fmts[1]['post_k'] and fmts[0]['post_fused'] and fmts[1]['post_fused']
    assert fmts[0]['post_sell'] == (sell == '1')
    assert rel(zs[0], zs[1]) < 1e-12
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs)
    assert rel(zs[0], h.apply(mo.seeded_rhs(s.N))) < APPLY_TOL


@pytest.mark.parametrize('dim,n,g,kw', [(3, 16, 1e6, dict()), (2, 64, 1e3, dict(maxit=2, presmooth_iter=2,
                                                                                   postsmooth_iter=2)),
                                        (3, 16, 1e4, dict(post_fusion=0))])
def test_half_symmetric_a0_bitwise(lib_built, monkeypatch, dim, n, g, kw):
    """Half-symmetric ELL-64 A_0 (upper blocks streamed, lower blocks read
    through their mirrors) sums every row in the full row's block order: the
    apply and the device PCG are bitwise those of full SELL-64 storage."""
    M = _mamg()
    set_opt('MAMG_SELL_MIN_ROWS', '1')
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    r = mo.seeded_rhs(s.N)
    outs, its = [], []
    for half in ('1', '0'):
        set_opt('MAMG_HALF', half)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **to_c(kw))
        f = B.level_format(0)
        assert f['sell'] != (half == '1') and f['half'] == (half == '1') and f['sym']
        outs.append(B * r)
        solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
        solver * r
        its.append(solver.residuals)
        B.close()
    h = mo.setup(A, mo.Params(num_functions=2, **oracle_kw(kw)), idofs=s.idofs)
    zo = h.apply(r)
    diff = np.flatnonzero(outs[0] != outs[1])
    assert diff.size == 0, dict(ndiff=int(diff.size), first=diff[:8].tolist(),
                                maxabs=float(np.abs(outs[0] - outs[1]).max()),
                                err_half=rel(outs[0], zo), err_full=rel(outs[1], zo))
    assert its[0] == its[1]
    assert rel(outs[0], zo) < APPLY_TOL


@pytest.mark.parametrize('bands', ['1', '2'])
def test_restriction_band_schedule_bitwise(lib_built, monkeypatch, bands):
    """The plane-band schedule of the level-0 restriction (coarse rows walked
    band by band through the planes on each XCD) only reorders workgroups:
    at 3-D n=128 the apply and the device PCG are bitwise those of the
    XCD-contiguous order (MAMG_R_BANDS=0)."""
    M = _mamg()
    s = M.problems.bidomain(3, 128, 1e6)
    A = s.scipy()
    r = mo.seeded_rhs(s.N)
    outs, its = [], []
    for b in (bands, '0'):
        set_opt('MAMG_R_BANDS', b)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        assert B.level_format(0)['r_bands'] == (b != '0')
        outs.append(B * r)
        solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
        solver * r
        its.append(solver.residuals)
        B.close()
    assert np.array_equal(outs[0], outs[1])
    assert its[0] == its[1]


@pytest.mark.parametrize('bands', ['1', '2'])
def test_half_band_schedule_bitwise(lib_built, monkeypatch, bands):
    """The band schedule of the half-symmetric kernel (rows walked plane band
    by plane band on each XCD) only reorders workgroups: at 3-D n=128 (where
    it engages) the apply and the device PCG are bitwise those of row order."""
    M = _mamg()
    s = M.problems.bidomain(3, 128, 1e6)
    A = s.scipy()
    r = mo.seeded_rhs(s.N)
    outs, its = [], []
    for b in (bands, '0'):
        set_opt('MAMG_HALF_BANDS', b)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        f = B.level_format(0)
        assert f['half'] and f['bands'] == (b != '0')
        outs.append(B * r)
        solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
        solver * r
        its.append(solver.residuals)
        B.close()
    assert np.array_equal(outs[0], outs[1])
    assert its[0] == its[1]


@pytest.mark.parametrize('kw', [dict(), dict(smoother='POLY'), dict(cycle_type='W', coarse_scaling=1),
                                dict(presmooth_iter=2, postsmooth_iter=2, maxit=2)])
def test_restriction_first_sweep_fused_bitwise(lib_built, monkeypatch, kw):
    """The coarse levels' first sweep x1 = W b written by the restriction's
    epilogue (EPI_YBD, one launch fewer per coarse level) is bitwise the
    separate bd2 launch: applies and the device PCG's history equal."""
    M = _mamg()
    s = M.problems.bidomain(3, 32, 1e6)
    A = s.scipy()
    r = mo.seeded_rhs(s.N)
    outs, its = [], []
    for f in ('2', '1', '0'):   # default (below level 0), every level, none
        set_opt('MAMG_FUSE_RBD', f)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **to_c(kw))
        outs.append(B * r)
        solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
        solver * r
        its.append(solver.residuals)
        B.close()
    for k in (1, 2):
        assert np.array_equal(outs[0], outs[k])
        assert its[0] == its[k]
    h = mo.setup(A, mo.Params(num_functions=2, **kw), idofs=s.idofs)
    assert rel(outs[0], h.apply(r)) < APPLY_TOL


def test_half_symmetric_rejects_nonsymmetric(lib_built, monkeypatch):
    """A_0 whose 2x2 blocks are symmetric but A_IJ != A_JI in one ulp: the
    mirror check rejects the half format (full SELL-64 is used) and the apply
    still matches the oracle."""
    M = _mamg()
    set_opt('MAMG_SELL_MIN_ROWS', '1')
    s = M.problems.bidomain(3, 8, 1e2)
    A = s.scipy().tocsr().copy()
    row = int(np.argmax(np.diff(A.indptr)[:s.nv]))      # an interior field-0 row
    k = next(k for k in range(A.indptr[row], A.indptr[row + 1]) if A.indices[k] != row
             and A.indices[k] < s.nv)
    A.data[k] = np.nextafter(A.data[k], np.inf)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    f = B.level_format(0)
    assert f['sell'] and not f['half']
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    assert rel(B * r, h.apply(r)) < APPLY_TOL
    B.close()


@pytest.mark.parametrize('dim,n,g,kw', [(3, 16, 1e6, dict()), (3, 16, 1e10, dict()),
                                        (2, 64, 1e3, dict(maxit=2, presmooth_iter=2, postsmooth_iter=2)),
                                        (3, 16, 1e4, dict(cycle_type='W')),
                                        (3, 8, 1e2, dict(post_fusion=0))])
def test_sell_layout_matches_oracle(lib_built, monkeypatch, dim, n, g, kw):
    """SELL-64 storage (one lane per node row; used for the level-0 operators
    at benchmark size) forced onto every short-row level of small problems:
    all epilogues, field-major x (maxit > 1, PCG), the fused post kernel."""
    set_opt('MAMG_SELL_MIN_ROWS', '1')
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **to_c(kw))
    h = mo.setup(A, mo.Params(num_functions=2, **oracle_kw(kw)), idofs=s.idofs)
    tol = APPLY_TOL if g < 1e8 else 1e-8
    for seed in (1234, 5):
        r = mo.seeded_rhs(s.N, seed)
        assert rel(B * r, h.apply(r)) < tol
    b = mo.seeded_rhs(s.N)
    solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)   # device PCG (A_0 SpMV)
    solver * b
    ref = mo.pcg(A, h, b, 1e-8, 500)
    assert len(solver.residuals) == len(ref.residuals)


def test_bsr2_spmv_and_pcg_field_major(lib_built):
    import torch
    M = _mamg()
    s = M.problems.bidomain(3, 16, 1e5)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    assert B.layout == 'bsr2'
    x = np.random.default_rng(9).standard_normal(s.N)
    y = torch.empty(s.N, dtype=torch.float64, device='cuda')
    B.spmv_device(torch.as_tensor(x).cuda(), y)
    torch.cuda.synchronize()
    assert rel(y.cpu().numpy(), A @ x) < 1e-14


def test_edge_cases(lib_built):
    M = _mamg()
    # coarsest immediately (n <= coarse_dof): pure dense solve
    A = mo.laplace1d(50)
    B = M.MetricAMG(A)
    r = mo.seeded_rhs(50)
    assert B.num_levels == 1
    assert rel(B * r, np.linalg.solve(A.toarray(), r)) < 1e-12
    # 1x1
    import scipy.sparse as sp
    B1 = M.MetricAMG(sp.csr_matrix(np.array([[4.0]])))
    assert abs((B1 * np.array([2.0]))[0] - 0.5) < 1e-15
    # isolated (identity) rows mixed with a Laplacian
    L = sp.block_diag([mo.laplace1d(400), sp.eye(30)]).tocsr()
    L.sort_indices()
    B2 = M.MetricAMG(L, coarse_dof=20)
    h = mo.setup(L, mo.Params(coarse_dof=20))
    r = mo.seeded_rhs(430)
    assert rel(B2 * r, h.apply(r)) < APPLY_TOL
    # bad vector size
    with pytest.raises(ValueError):
        B2 * np.ones(3)


def test_multiple_handles_and_graph_cache(lib_built):
    import torch
    M = _mamg()
    s1 = M.problems.bidomain(2, 32, 1.0)
    s2 = M.problems.bidomain(3, 8, 1e6)
    B1 = M.MetricAMG(s1.scipy(), s1.W, idofs=s1.idofs, num_functions=2)
    B2 = M.MetricAMG(s2.scipy(), s2.W, idofs=s2.idofs, num_functions=2)
    r1 = torch.as_tensor(mo.seeded_rhs(s1.N)).cuda()
    r2 = torch.as_tensor(mo.seeded_rhs(s2.N)).cuda()
    outs = []
    z1 = torch.empty_like(r1)
    for _ in range(5):                     # many distinct (r, z) pairs + replays
        B1.apply_device(r1, z1)
        outs.append(z1.clone())
        B2.matvec(r2)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])     # deterministic replays (bitwise)
    B1.close()
    B2.close()


def test_large_properties_3d(lib_built):
    """bidomain_3d nrefs=5 (BASELINE config 3, N = 4.29M): symmetry,
    linearity, positivity, determinism of the device apply."""
    import torch
    M = _mamg()
    s = M.problems.bidomain(3, 128, 1e6)
    B = M.MetricAMG(s, s.W, idofs=s.idofs, num_functions=2)
    g = torch.Generator(device='cuda').manual_seed(5)
    r = torch.rand(s.N, dtype=torch.float64, device='cuda', generator=g) * 2 - 1
    q = torch.rand(s.N, dtype=torch.float64, device='cuda', generator=g) * 2 - 1
    Br, Bq = B.matvec(r), B.matvec(q)
    a, b = torch.dot(Br, q).item(), torch.dot(r, Bq).item()
    assert abs(a - b) <= 1e-9 * (abs(a) + abs(b))
    assert torch.dot(Br, r).item() > 0
    lin = B.matvec(2.0 * r + q)
    assert (torch.linalg.norm(lin - (2.0 * Br + Bq)) / torch.linalg.norm(lin)).item() < 1e-12
    assert torch.equal(B.matvec(r), Br)


def test_host_apply_after_queued_device_apply(lib_built):
    """A device-pointer apply queued on torch's stream and a host-pointer
    apply (handle stream) right after it share the handle's scratch vectors:
    the handle serializes them, both equal the oracle."""
    import torch
    M = _mamg()
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs)
    r1, r2 = mo.seeded_rhs(s.N, 1), mo.seeded_rhs(s.N, 2)
    big = torch.randn(4096, 4096, device='cuda')
    for _ in range(3):
        big = big @ big * 1e-3                  # keep torch's stream busy first
    zt = B.matvec(torch.as_tensor(r1).cuda())
    z2 = B * r2                                 # host apply, immediately
    torch.cuda.synchronize()
    assert rel(zt.cpu().numpy(), h.apply(r1)) < APPLY_TOL
    assert rel(z2, h.apply(r2)) < APPLY_TOL


def test_graph_cache_eviction(lib_built):
    """More than 16 distinct (r, z) buffer pairs: the graph cache evicts
    (after the handle's queued work finished) and every result is right."""
    import torch
    M = _mamg()
    s = M.problems.bidomain(2, 32, 1e3)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs)
    rs = [mo.seeded_rhs(s.N, k) for k in range(24)]
    outs = [B.matvec(torch.as_tensor(r).cuda()) for r in rs]      # fresh z each time
    torch.cuda.synchronize()
    for r, z in zip(rs, outs):
        assert rel(z.cpu().numpy(), h.apply(r)) < APPLY_TOL


def test_device_conjgrad_requires_own_operator(lib_built):
    M = _mamg()
    s = M.problems.bidomain(2, 16, 1e2)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    with pytest.raises(ValueError):
        M.ConjGrad(A.copy(), precond=B, device=True) * mo.seeded_rhs(s.N)


def test_k_block_layouts_bitwise(lib_built, monkeypatch):
    """The K values stored one 32-byte block per SELL slot (default) or as two
    16-byte streams (MAMG_POST_K=2, kpost_kernel SPL): the same sums, so the
    apply and the device PCG are bitwise equal."""
    import torch
    M = _mamg()
    set_opt('MAMG_SELL_MIN_ROWS', '1')
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    r = torch.as_tensor(mo.seeded_rhs(s.N)).cuda()
    zs, its = [], []
    for mode in ('3', '2'):
        set_opt('MAMG_POST_K', mode)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        assert B.level_format(0)['post_sell']
        zs.append(B.matvec(r))
        cg = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
        x = cg * mo.seeded_rhs(s.N)
        its.append((len(cg.residuals), np.asarray(x.cpu() if hasattr(x, 'cpu') else x)))
        torch.cuda.synchronize()
        B.close()
    assert torch.equal(zs[0], zs[1])
    assert its[0][0] == its[1][0] and np.array_equal(its[0][1], its[1][1])
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs)
    assert rel(zs[1].cpu().numpy(), h.apply(mo.seeded_rhs(s.N))) < APPLY_TOL


@pytest.mark.parametrize('dim,n,g', [(3, 16, 1e6), (3, 32, 1e6), (2, 128, 1e4)])
def test_k_col16_bitwise(lib_built, dim, n, g):
    """Level-0 K's columns as 16-bit offsets from a per-slice base (round 6,
    MAMG_K_COL16=1, the default): the kernel adds the base back, so the apply
    and the device PCG are bitwise those of the 32-bit columns, and = the
    oracle."""
    import torch
    M = _mamg()
    set_opt('MAMG_SELL_MIN_ROWS', '1')
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    r = torch.as_tensor(mo.seeded_rhs(s.N)).cuda()
    zs, its = [], []
    for c16 in ('0', '1'):
        set_opt('MAMG_K_COL16', c16)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        assert B.level_format(0)['post_sell'] and B.level_format(0)['k_col16'] == (c16 == '1')
        zs.append(B.matvec(r))
        cg = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
        x = cg * mo.seeded_rhs(s.N)
        its.append((len(cg.residuals), np.asarray(x.cpu() if hasattr(x, 'cpu') else x)))
        torch.cuda.synchronize()
        B.close()
    assert torch.equal(zs[0], zs[1])
    assert its[0][0] == its[1][0] and np.array_equal(its[0][1], its[1][1])
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs)
    assert rel(zs[1].cpu().numpy(), h.apply(mo.seeded_rhs(s.N))) < APPLY_TOL


# MAMG_K_VARIANT exists only in the diagnosis build: these run in a child
# process that loads it (tests/test_gpu_poison.py)
needs_diag = pytest.mark.skipif(not __import__('conftest').diag_loaded(),
                                reason='diagnosis build only (MAMG_LIB=libmamg_diag.so; run by test_gpu_poison.py)')


@needs_diag
@pytest.mark.parametrize('variant', ['0', '1', '2'])
def test_k_kernel_variants(lib_built, monkeypatch, variant):
    """The level-0 K kernel with 2 lanes per row (default), 1 lane (round 2's
    sell2_kernel) or 4 lanes: the same operator up to the order of a row's
    partial sums (1e-14), each = the oracle; the eager (time_apply) launches
    give the graph apply's bits, and the operators re-homed after the setup
    give the bits of the un-moved ones."""
    import torch
    M = _mamg()
    set_opt('MAMG_SELL_MIN_ROWS', '1')
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    r = torch.as_tensor(mo.seeded_rhs(s.N)).cuda()
    monkeypatch.setenv('MAMG_K_VARIANT', '1')
    B1 = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    z1 = B1.matvec(r)
    torch.cuda.synchronize()
    monkeypatch.setenv('MAMG_K_VARIANT', variant)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    assert B.level_format(0)['post_sell']
    z = B.matvec(r)
    zz = torch.empty_like(z)
    B.time_apply(r, zz, 1, 0)
    torch.cuda.synchronize()
    assert torch.equal(zz, z)
    set_opt('MAMG_REHOME', '0')
    B0 = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    z0 = B0.matvec(r)
    torch.cuda.synchronize()
    # each handle against the oracle first, so that a failure names the handle
    zo = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs).apply(mo.seeded_rhs(s.N))
    errs = {k: rel(v.cpu().numpy(), zo) for k, v in (('B1', z1), ('B', z), ('B relayout', zz), ('B0', z0))}
    assert max(errs.values()) < APPLY_TOL, (errs, B.kregion)
    assert torch.equal(z0, z), (rel(z0.cpu().numpy(), z.cpu().numpy()), B.kregion)
    assert rel(z.cpu().numpy(), z1.cpu().numpy()) < 1e-14
    for b in (B, B0, B1):
        b.close()


@needs_diag
@pytest.mark.parametrize('variant', ['0', '1', '2'])
def test_k_row_sort_bitwise(lib_built, monkeypatch, variant):
    """Level-0 K with its rows sorted by length inside each SELL slice
    (MAMG_K_SORT=1, the default; sort_sell_slices) gives the bits of row
    order, for the two-lane, one-lane and four-lane K kernels, on the graph
    apply and the eager launches, and equals the oracle."""
    import torch
    M = _mamg()
    set_opt('MAMG_SELL_MIN_ROWS', '1')
    monkeypatch.setenv('MAMG_K_VARIANT', variant)
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    r = torch.as_tensor(mo.seeded_rhs(s.N)).cuda()
    zs = []
    for srt in ('0', '1'):
        set_opt('MAMG_K_SORT', srt)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        assert B.level_format(0)['post_sell']
        z = B.matvec(r)
        zz = torch.empty_like(z)
        B.time_apply(r, zz, 1, 0)
        torch.cuda.synchronize()
        assert torch.equal(zz, z)
        zs.append(z.clone())
        B.close()
    assert torch.equal(zs[0], zs[1])
    zo = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs).apply(mo.seeded_rhs(s.N))
    assert rel(zs[1].cpu().numpy(), zo) < APPLY_TOL


@pytest.mark.parametrize('dim,n,g,kw', [(3, 16, 1e6, dict()), (2, 64, 1e4, dict(smoother='POLY')),
                                        (3, 16, 1e6, dict(presmooth_iter=2, postsmooth_iter=2))])
def test_coarse_multilane_sell(lib_built, monkeypatch, dim, n, g, kw):
    """Coarse levels' A and K stored SELL-64 with several lanes per row
    (msell_kernel; MAMG_MSELL_MIN_ROWS lowered so every level takes it) equal
    the lane-group BSR kernels up to summation order, and the oracle."""
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    r = mo.seeded_rhs(s.N)
    zs = []
    for rows in ('1', str(1 << 30)):
        set_opt('MAMG_MSELL_MIN_ROWS', rows)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **to_c(kw))
        assert B.level_format(1)['sell'] == (rows == '1')
        zs.append(B * r)
        B.close()
    assert rel(zs[0], zs[1]) < 1e-13
    h = mo.setup(A, mo.Params(num_functions=2, **kw), idofs=s.idofs)
    assert rel(zs[0], h.apply(r)) < APPLY_TOL


def test_pcg_graph_reused_across_solves(lib_built):
    """mamg_pcg_device keeps the captured iteration graph per (x, maxiter):
    repeated solves (driver loops, gamma sweeps) into the same x give the same
    iterations and bits as the first, and a different maxiter gets its own."""
    import torch
    M = _mamg()
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    b = torch.as_tensor(mo.seeded_rhs(s.N)).cuda()
    x = torch.zeros_like(b)
    outs = []
    for maxiter in (500, 500, 7, 500):
        x.zero_()
        cg = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=maxiter)
        cg.solve_device(b, x)
        torch.cuda.synchronize()
        outs.append((list(cg.residuals), x.clone()))
    assert outs[0][0] == outs[1][0] == outs[3][0] and len(outs[2][0]) == 8
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][1], outs[3][1])
    ref = mo.pcg(A, mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs), mo.seeded_rhs(s.N), 1e-8, 500)
    assert len(outs[0][0]) == len(ref.residuals)
