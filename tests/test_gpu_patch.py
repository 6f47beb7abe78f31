"""GPU parity of the multiplicative node-patch Schwarz smoother
(Schwarz_type SCHWARZ_PATCHES: the reference's level-0 symmetric
multiplicative Schwarz on the seeds' overlapping 1-ring blocks,
/root/reference/src/amg_parameters.py:83-87, src/utils.py:84) against the CPU
oracle (mamg_oracle.Patches: distance-3 colouring, Gauss-Jordan patch
inverses, colour-ordered sweeps).

Tolerances as tests/test_gpu_gs.py: one apply to 1e-10 relative (colouring,
order and patch inverses are exact; only the residual summation order
differs), PCG iteration count equal to the oracle's, residuals within 1e-6.
"""
import numpy as np
import pytest

import mamg_oracle as mo
from conftest import set_opt

pytestmark = pytest.mark.gpu

PATCHES = 6


def _mamg():
    import metric_amg_examples_amd as M
    return M


def to_c(kw):
    c = dict(kw, Schwarz_type=PATCHES)
    if 'smoother' in c:
        c['smoother'] = {'SGS': 11, 'GS': 10, 'POLY': 12}[c['smoother']]
    if 'cycle_type' in c:
        c['cycle_type'] = {'V': 1, 'W': 2}[c['cycle_type']]
    if 'AMG_type' in c:
        c['AMG_type'] = {'SA': 2, 'UA': 1}[c['AMG_type']]
    if 'aggregation_type' in c:
        c['aggregation_type'] = {'MIS': 2, 'HEM': 5}[c['aggregation_type']]
    return c


def rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


CASES = [
    (3, 8, 1e6, dict()),
    (3, 16, 1e6, dict()),
    (2, 32, 1.0, dict()),
    (2, 64, 1e6, dict(coarse_scaling=1)),
    (3, 16, 1e4, dict(smoother='SGS', coarse_scaling=1)),
    (3, 8, 1e2, dict(smoother='POLY')),
    (3, 16, 1e6, dict(cycle_type='W', presmooth_iter=2, postsmooth_iter=2)),
    # the reference's metric_schwarz family with its own level-0 Schwarz:
    # UA + parallel HEM + W-cycle + SGS + coarse scaling + node patches
    (3, 16, 1e6, dict(smoother='SGS', coarse_scaling=1, cycle_type='W', AMG_type='UA', aggregation_type='HEM')),
]


@pytest.mark.parametrize('setup', ['host', 'gpu'])
@pytest.mark.parametrize('dim,n,g,kw', CASES)
def test_patch_apply_matches_oracle(lib_built, dim, n, g, kw, setup):
    import torch
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup=setup, **to_c(kw))
    assert B.setup_path == setup, B.setup_path
    h = mo.setup(A, mo.Params(num_functions=2, Schwarz_type=PATCHES, **kw), idofs=s.idofs)
    assert B.num_levels == len(h.levels)
    for seed in (1234, 7):
        r = mo.seeded_rhs(s.N, seed)
        zo = h.apply(r)
        z = B * r
        assert rel(z, zo) < 1e-10
        zt = B.matvec(torch.as_tensor(r).cuda())
        torch.cuda.synchronize()
        assert rel(zt.cpu().numpy(), zo) < 1e-10


@pytest.mark.parametrize('dim,n,g', [(3, 16, 1e6), (2, 64, 1e4), (3, 8, 1e10), (3, 16, 1e10)])
def test_patch_pcg_matches_oracle(lib_built, dim, n, g):
    """Device PCG with the node-patch profile against the oracle's PCG:
    the same iteration count; every residual sqrt(<r, Br>) within rtol 1e-6
    (gamma <= 1e6) or 1e-4 (gamma = 1e10), or within 1e-12 of the first
    residual; the true relative residual ||b - Ax|| / ||b|| of both solutions
    at the level the oracle's own solution reaches, and the solutions equal in
    the energy of A to 1e-6 of b.  Why 1e-4 at gamma = 1e10: the patch
    matrices' condition numbers are ~gamma, so any two inverses computed in a
    different operation order (the oracle's scalar Gauss-Jordan, the device's
    matrix-core block sweep, patch_inv3_kernel) differ by ~gamma * eps = 1e-6
    relative, and the Krylov residuals inherit it (measured 8.7e-6 at the
    4th residual); the scalar kernels (MAMG_PATCH_INV=1, 2) repeat the
    oracle's order and stay within 1e-6 (round 5)."""
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    b = mo.seeded_rhs(s.N)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, Schwarz_type=PATCHES)
    solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
    x = solver * b
    x = x.cpu().numpy() if hasattr(x, 'cpu') else np.asarray(x)
    h = mo.setup(A, mo.Params(num_functions=2, Schwarz_type=PATCHES), idofs=s.idofs)
    ref = mo.pcg(A, h, b, 1e-8, 500)
    assert len(solver.residuals) == len(ref.residuals)
    res, rres = np.asarray(solver.residuals), np.asarray(ref.residuals)
    assert res[-1] <= 1e-8 and rres[-1] <= 1e-8
    rtol = 1e-6 if g <= 1e6 else 1e-4
    assert np.allclose(res, rres, rtol=rtol, atol=1e-12 * rres[0]), np.abs(res - rres) / rres
    bn = np.linalg.norm(b)
    rel_true, rel_true_o = np.linalg.norm(b - A @ x) / bn, np.linalg.norm(b - A @ ref.x) / bn
    assert rel_true <= max(2.0 * rel_true_o, 1e-12), (rel_true, rel_true_o)
    assert np.linalg.norm(A @ (x - ref.x)) <= 1e-6 * bn


def test_patch_cycle_symmetric_and_deterministic(lib_built):
    """Forward + backward colour sweeps make the cycle a symmetric operator;
    two graph replays give identical bits (no races inside a colour)."""
    import torch
    M = _mamg()
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, Schwarz_type=PATCHES)
    r1 = torch.as_tensor(mo.seeded_rhs(s.N, 1)).cuda()
    r2 = torch.as_tensor(mo.seeded_rhs(s.N, 2)).cuda()
    z1, z2 = B.matvec(r1), B.matvec(r2)
    z1b = B.matvec(r1)
    torch.cuda.synchronize()
    a = float(torch.dot(r2, z1))
    c = float(torch.dot(r1, z2))
    assert abs(a - c) <= 1e-12 * abs(a)
    assert torch.equal(z1, z1b)


def test_patch_bidomain_3d_nrefs4(lib_built):
    """A larger 3-D case (n = 64, 550K dofs) on the GPU setup: the device PCG
    equals the host loop (same preconditioner, graph vs host-staged applies)."""
    M = _mamg()
    s = M.problems.bidomain(3, 64, 1e6)
    A = s.scipy()
    b = mo.seeded_rhs(s.N)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, Schwarz_type=PATCHES, setup='gpu')
    dev = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
    dev * b
    host = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500, device=False)
    host * b
    assert len(dev.residuals) == len(host.residuals) < 100
    assert np.allclose(dev.residuals, host.residuals, rtol=1e-6, atol=0)


def _oracle_params(d, **kw):
    """A reference parameter dict (src/amg_parameters.py) as oracle Params."""
    M = _mamg()
    P = M.parameters
    return mo.Params(
        AMG_type={P.UA_AMG: 'UA', P.SA_AMG: 'SA'}[d['AMG_type']],
        cycle_type={P.V_CYCLE: 'V', P.W_CYCLE: 'W'}[d['cycle_type']],
        aggregation_type={P.MIS: 'MIS', P.HEM: 'HEM', P.VMB: 'VMB'}[d['aggregation_type']],
        smoother={P.SMOOTHER_SGS: 'SGS', P.SMOOTHER_GS: 'GS', P.SMOOTHER_JACOBI_RHO: 'JACOBI_RHO'}[d['smoother']],
        max_levels=d['max_levels'], maxit=d['maxit'], relaxation=d['relaxation'],
        presmooth_iter=d['presmooth_iter'], postsmooth_iter=d['postsmooth_iter'], coarse_dof=d['coarse_dof'],
        strong_coupled=d['strong_coupled'], coarse_scaling=d['coarse_scaling'],
        Schwarz_levels=d['Schwarz_levels'], Schwarz_mmsize=d.get('Schwarz_mmsize', 100),
        Schwarz_maxlvl=d.get('Schwarz_maxlvl', 1), Schwarz_type=d.get('Schwarz_type', 4), **kw)


@pytest.mark.parametrize('setup', ['host', 'gpu'])
def test_reference_preset_metric_schwarz(lib_built, setup):
    """metricAMG(A, W, idofs, parameters=parameters_metric_schwarz) -- the
    reference's own call (src/bidomain_3d.py:138-147, src/utils.py:86) with
    its preset verbatim (src/amg_parameters.py:67-89: UA, HEM, W-cycle, SGS,
    coarse scaling, SCHWARZ_SYMMETRIC on the seeds' 1-rings) -- runs the
    overlapping node patches on level 0 (num_functions from W) and equals the
    oracle's restatement of the same algorithm: one apply to 1e-10, the PCG
    iteration count and residuals."""
    import torch
    M = _mamg()
    P = M.parameters
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    B = M.metricAMG(A, s.W, idofs=s.idofs, parameters=P.parameters_metric_schwarz, setup=setup)
    assert B.setup_path == setup, B.setup_path
    assert B.effective_params['Schwarz_type'] == P.SCHWARZ_PATCHES
    assert B.effective_params['num_functions'] == 2
    assert B.level_format(0)['patches'] and B.level_format(1)['gs']
    h = mo.setup(A, _oracle_params(P.parameters_metric_schwarz, num_functions=2), idofs=s.idofs)
    assert h.levels[0].patches is not None and B.num_levels == len(h.levels)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    assert rel(B * r, zo) < 1e-10
    zt = B.matvec(torch.as_tensor(r).cuda())
    torch.cuda.synchronize()
    assert rel(zt.cpu().numpy(), zo) < 1e-10
    solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
    solver * r
    ref = mo.pcg(A, h, r, 1e-8, 500)
    assert len(solver.residuals) == len(ref.residuals)
    assert np.allclose(solver.residuals, ref.residuals, rtol=1e-6, atol=0)


@pytest.mark.parametrize('setup', ['gpu', 'host'])
def test_reference_preset_standard_vmb(lib_built, setup):
    """metricAMG(A, W, parameters=parameters_standard): the reference's
    standard preset verbatim (src/amg_parameters.py:16-36: UA, sequential
    Vanek-Mandel-Brezina aggregation, W-cycle, SGS, coarse scaling, no
    Schwarz).  The GPU setup runs the sequential aggregation step on the host
    (on the strong graph it built) and everything else on the device; either
    setup's apply equals the oracle's restatement to 1e-10, with the same PCG
    iteration count and residuals."""
    M = _mamg()
    P = M.parameters
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    B = M.metricAMG(A, s.W, idofs=s.idofs, parameters=P.parameters_standard, setup=setup)
    assert B.setup_path == setup, B.setup_path
    assert B.effective_params['aggregation_type'] == P.VMB
    assert B.level_format(1)['gs']
    h = mo.setup(A, _oracle_params(P.parameters_standard, num_functions=2), idofs=s.idofs)
    assert B.num_levels == len(h.levels)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    assert rel(B * r, zo) < 1e-10
    solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
    solver * r
    ref = mo.pcg(A, h, r, 1e-8, 500)
    assert len(solver.residuals) == len(ref.residuals)
    assert np.allclose(solver.residuals, ref.residuals, rtol=1e-6, atol=0)


def test_patches_refused_on_the_csr_layout(lib_built):
    """Node patches run only in the BSR2 layout: with seeds that leave the
    level-0 seed blocks not node-aligned (u1 of the even nodes, u0 of the odd
    ones, gamma = 1: a u0 dof's strongest seed neighbour is another node's),
    the hierarchy takes the CSR layout, and both setups refuse instead of
    running seed-block Jacobi under the patch name."""
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(2, 16, 1.0)
    nv = s.nv
    idofs = np.array([nv + I if I % 2 == 0 else I for I in range(nv)], np.int32)
    for setup in ('host', 'gpu'):
        with pytest.raises(M._lib.MamgError) as ei:
            M.MetricAMG(s.scipy(), s.W, idofs=idofs, num_functions=2, setup=setup,
                        Schwarz_type=M.parameters.SCHWARZ_PATCHES)
        assert ei.value.code == -4 and 'BSR2' in str(ei.value), (setup, str(ei.value))


@pytest.mark.parametrize('dim,n', [(3, 16), (3, 32), (2, 64)])
def test_patch_inverse_kernels_bitwise(lib_built, dim, n):
    """the node-patch inverses two patches per wave, in place
    (patch_inv2_kernel: lane k takes over identity column k at pivot k, the
    rows' block searches interleaved) perform the round-5 kernel's operations
    on the same values (MAMG_PATCH_INV=1: one patch per wave, the augmented
    [A_p | I] in 64 lanes), so the applies and the PCG iterates are bitwise
    equal; on the verbatim preset too (UA + HEM + W + SGS + scaling)."""
    import torch
    M = _mamg()
    s = M.problems.bidomain(dim, n, 1e6)
    A = s.scipy()
    r = torch.as_tensor(mo.seeded_rhs(s.N)).cuda()
    for prm in (dict(num_functions=2, Schwarz_type=PATCHES),
                dict(parameters=M.parameters.parameters_metric_schwarz)):
        zs, xs = [], []
        for v in ('1', '2'):
            set_opt('MAMG_PATCH_INV', v)
            B = M.MetricAMG(A, s.W, idofs=s.idofs, setup='gpu', **prm)
            assert B.level_format(0)['patches']
            zs.append(B.matvec(r).clone())
            B._Aop = A
            cg = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
            xs.append((list(cg.residuals) if cg.solve_device(r) is not None else None, cg.residuals))
            torch.cuda.synchronize()
            B.close()
        assert torch.equal(zs[0], zs[1])
        assert xs[0][1] == xs[1][1]


@pytest.mark.gpu
@pytest.mark.parametrize('dim,n', [(3, 8), (3, 16), (2, 32)])
def test_patch_inverse_matrix_cores(lib_built, dim, n):
    """the patch inverses by the f64 matrix-core block sweep
    (patch_inv3_kernel, MAMG_PATCH_INV=3, the default) against the scalar
    Gauss-Jordan kernel (MAMG_PATCH_INV=2): a different rounding, so not
    bitwise -- the applies agree to 1e-10, the PCG takes the same
    iterations and its residual history agrees to 1e-6; the oracle parity of
    the default path is test_patch_apply_matches_oracle."""
    import torch
    M = _mamg()
    s = M.problems.bidomain(dim, n, 1e6)
    A = s.scipy()
    r = torch.as_tensor(mo.seeded_rhs(s.N)).cuda()
    for prm in (dict(num_functions=2, Schwarz_type=PATCHES),
                dict(parameters=M.parameters.parameters_metric_schwarz)):
        zs, hs = [], []
        for v in ('2', '3'):
            set_opt('MAMG_PATCH_INV', v)
            B = M.MetricAMG(A, s.W, idofs=s.idofs, setup='gpu', **prm)
            assert B.level_format(0)['patches']
            zs.append(B.matvec(r).clone())
            B._Aop = A
            cg = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
            cg.solve_device(r)
            hs.append(list(cg.residuals))
            torch.cuda.synchronize()
            B.close()
        assert float(torch.linalg.norm(zs[0] - zs[1]) / torch.linalg.norm(zs[0])) < 1e-10
        assert len(hs[0]) == len(hs[1])
        assert all(abs(a - b) <= 1e-6 * abs(a) for a, b in zip(hs[0], hs[1]))
