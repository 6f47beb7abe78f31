"""GPU parity of the multicolour node-block Gauss-Seidel smoothers and the
coarse-grid correction scaling (the reference's SMOOTHER_SGS and
coarse_scaling ON, /root/reference/src/amg_parameters.py:72,78) against the
CPU oracle (mamg_oracle: jp_colouring, Level.gs_sweep, coarse_scale).

Tolerances as tests/test_gpu.py: one apply to 1e-10 relative (the colouring,
permutation and block inverses are exact; only SpMV summation order differs),
PCG iteration count equal to the oracle's and residuals within 1e-6.
"""
import numpy as np
import pytest

import mamg_oracle as mo
from conftest import set_opt

pytestmark = pytest.mark.gpu

SMO = {'SGS': 11, 'GS': 10}


def _mamg():
    import metric_amg_examples_amd as M
    return M


def to_c(kw):
    c = dict(kw)
    if 'smoother' in c:
        # the level-0 seed blocks take the level smoother (SCHWARZ_SEED_BLOCKS)
        c['Schwarz_type'] = 7
        c['smoother'] = SMO[c['smoother']]
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
    (2, 32, 1.0, dict(smoother='SGS')),
    (2, 64, 1e6, dict(smoother='SGS', coarse_scaling=1)),
    (3, 8, 1e6, dict(smoother='GS')),
    (3, 16, 1e6, dict(smoother='SGS')),
    (3, 16, 1e6, dict(smoother='SGS', coarse_scaling=1, cycle_type='W')),
    (3, 16, 1e10, dict(smoother='SGS', coarse_scaling=1)),
    (3, 16, 1e2, dict(smoother='GS', presmooth_iter=2, postsmooth_iter=2)),
    (3, 16, 1e4, dict(coarse_scaling=1)),                      # Jacobi + scaling (K post)
    (2, 32, 1e3, dict(coarse_scaling=1, cycle_type='W')),
    # the reference's metric_mono family (src/amg_parameters.py:67-89) on the GPU:
    # UA + parallel HEM + W-cycle + SGS + coarse scaling
    (3, 16, 1e6, dict(smoother='SGS', coarse_scaling=1, cycle_type='W', AMG_type='UA', aggregation_type='HEM')),
    (2, 64, 1e4, dict(smoother='SGS', coarse_scaling=1, cycle_type='W', AMG_type='UA', aggregation_type='HEM')),
]


@pytest.mark.parametrize('setup', ['host', 'gpu'])
@pytest.mark.parametrize('dim,n,g,kw', CASES)
def test_gs_apply_matches_oracle(lib_built, dim, n, g, kw, setup):
    import torch
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup=setup, **to_c(kw))
    assert B.setup_path == setup, B.setup_path
    h = mo.setup(A, mo.Params(num_functions=2, **kw), idofs=s.idofs)
    assert B.num_levels == len(h.levels)
    tol = 1e-10 if g < 1e8 else 1e-8
    for seed in (1234, 7):
        r = mo.seeded_rhs(s.N, seed)
        zo = h.apply(r)
        z = B * r
        assert rel(z, zo) < tol
        zt = B.matvec(torch.as_tensor(r).cuda())
        torch.cuda.synchronize()
        assert rel(zt.cpu().numpy(), zo) < tol


@pytest.mark.parametrize('dim,n,g,kw', [
    (3, 16, 1e6, dict(smoother='SGS')),
    (3, 16, 1e6, dict(smoother='SGS', coarse_scaling=1)),
    (2, 128, 1e4, dict(smoother='SGS')),
    (3, 32, 1.0, dict(smoother='GS')),
])
def test_gs_pcg_matches_oracle(lib_built, dim, n, g, kw):
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    b = mo.seeded_rhs(s.N)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **to_c(kw))
    solver = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
    x = solver * b
    h = mo.setup(A, mo.Params(num_functions=2, **kw), idofs=s.idofs)
    ref = mo.pcg(A, h, b, 1e-8, 500)
    assert len(solver.residuals) == len(ref.residuals)
    assert np.allclose(solver.residuals, ref.residuals, rtol=1e-6, atol=0)
    assert rel(x, ref.x) < 1e-6


def test_sgs_symmetric_and_deterministic(lib_built):
    """SGS V-cycle (no scaling) is a symmetric linear operator; two graph
    replays give identical bits."""
    import torch
    M = _mamg()
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, smoother=SMO['SGS'], Schwarz_type=7)
    r1 = torch.as_tensor(mo.seeded_rhs(s.N, 1)).cuda()
    r2 = torch.as_tensor(mo.seeded_rhs(s.N, 2)).cuda()
    z1, z2 = B.matvec(r1), B.matvec(r2)
    z1b = B.matvec(r1)
    torch.cuda.synchronize()
    a = float(torch.dot(r2, z1))
    c = float(torch.dot(r1, z2))
    assert abs(a - c) <= 1e-12 * abs(a)
    assert torch.equal(z1, z1b)



@pytest.mark.parametrize('dim,n,g,kw', [
    (3, 16, 1e6, dict(smoother='SGS', coarse_scaling=1, cycle_type='W', AMG_type='UA', aggregation_type='HEM')),
    (3, 32, 1e6, dict(smoother='SGS', coarse_scaling=1, cycle_type='W', AMG_type='UA', aggregation_type='HEM')),
    (2, 64, 1e4, dict(smoother='SGS', coarse_scaling=1, cycle_type='W')),
    (3, 16, 1e6, dict(smoother='SGS')),
])
def test_coarse_tail_equals_launches(lib_built, monkeypatch, dim, n, g, kw):
    """The coarse tail (one 1024-thread workgroup runs the whole cycle below
    tail_level, device.hip tail_kernel) equals the launch-by-launch cycle up
    to FMA contraction (1e-13) and the oracle (1e-10): SGS colour sweeps,
    coarse scaling, W-cycle second visits, the dense coarsest solve."""
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    r = mo.seeded_rhs(s.N)
    zs = []
    # the whole cycle below level 1 in the tail, no tail, the default tail
    # level with and without its register-resident operators (TOp.res)
    for nodes, res in (('100000000', None), ('0', None), (None, None), (None, '0')):
        set_opt('MAMG_TAIL_NODES', nodes)
        set_opt('MAMG_TAIL_RES', res)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **to_c(kw))
        zs.append(B * r)
        B.close()
    for z in zs[:1] + zs[2:]:
        assert rel(z, zs[1]) < 1e-13
    h = mo.setup(A, mo.Params(num_functions=2, **kw), idofs=s.idofs)
    assert rel(zs[0], h.apply(r)) < 1e-10
