"""Multi-GPU apply on one GPU: P rank handles in lockstep with device-copy
exchanges (virtual communicator: same counts/offsets as the RCCL path), and a
real 1-rank RCCL communicator.  The gathered z must equal the single-rank
oracle apply (fp64, 1e-10)."""
import numpy as np
import pytest

import mamg_oracle as mo
from conftest import set_opt

pytestmark = pytest.mark.gpu


def _gather(s, handles, zs):
    z = np.zeros(s.N)
    for h, zl in zip(handles, zs):
        zl = zl.cpu().numpy()
        z[h.o0:h.o1] = zl[:h.nloc]
        z[s.nv + h.o0:s.nv + h.o1] = zl[h.nloc:]
    return z


@pytest.mark.parametrize('dim,n,g,P,rep', [(3, 16, 1e4, 2, 100), (3, 16, 1e4, 3, 100),
                                           (3, 16, 1e6, 4, 10 ** 6), (2, 64, 1.0, 4, 100),
                                           (3, 32, 1e6, 8, 1000)])
def test_virtual_ranks_match_oracle(lib_built, dim, n, g, P, rep):
    import torch
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(dim, n, g)
    h = mo.setup(s.scipy(), mo.Params(num_functions=2), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=rep,
                          num_functions=2) for p in range(P)]
    rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
    zs = [torch.zeros_like(x) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, zs)
    torch.cuda.synchronize()
    z = _gather(s, hs, zs)
    assert np.linalg.norm(z - zo) / np.linalg.norm(zo) < 1e-10
    # repeated application is deterministic
    zs2 = [torch.zeros_like(x) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, zs2)
    torch.cuda.synchronize()
    for a, b in zip(zs, zs2):
        assert torch.equal(a, b)


@pytest.mark.parametrize('problem,kw,P', [
    ('bidomain', dict(smoother='POLY'), 3), ('bidomain', dict(smoother='POLY', poly_degree=3), 8),
    ('emi', {}, 2), ('emi', {}, 3), ('emi', dict(smoother='POLY'), 8), ('emi2d', dict(smoother='POLY'), 4)])
def test_virtual_ranks_poly_and_emi(lib_built, problem, kw, P):
    """The Chebyshev smoother (halo before every extra step; K built with the
    first post step's smoother) and EMI (interface seeds with node-aligned
    blocks, Schwarz_maxlvl 0: BSR2 + GPU setup on every rank) on P virtual
    ranks equal the single-rank oracle apply (BASELINE config 4's operator)."""
    import torch
    import metric_amg_examples_amd as M
    ckw = dict(kw)
    if problem.startswith('emi'):
        s = M.problems.emi(3, 16, 1e6) if problem == 'emi' else M.problems.emi(2, 64, 1e6)
        kw = dict(kw, Schwarz_maxlvl=0)
        ckw['Schwarz_maxlvl'] = 0
    else:
        s = M.problems.bidomain(3, 16, 1e6)
    if ckw.get('smoother') == 'POLY':
        ckw['smoother'] = 12
    h = mo.setup(s.scipy(), mo.Params(num_functions=2, **kw), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=100,
                          num_functions=2, **ckw) for p in range(P)]
    rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
    zs = [torch.zeros_like(x) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, zs)
    torch.cuda.synchronize()
    z = _gather(s, hs, zs)
    assert np.linalg.norm(z - zo) / np.linalg.norm(zo) < 1e-10
    for hh in hs:
        hh.close()


@pytest.mark.parametrize('kw,P,rep', [
    (dict(cycle_type='W'), 2, 100), (dict(cycle_type='W'), 3, 1), (dict(coarse_scaling=1), 3, 100),
    (dict(coarse_scaling=1), 8, 1), (dict(cycle_type='W', coarse_scaling=1, presmooth_iter=2, postsmooth_iter=2), 3, 1),
    (dict(smoother='POLY', coarse_scaling=1, cycle_type='W'), 8, 100),
    (dict(AMG_type='UA', aggregation_type='HEM', cycle_type='W', coarse_scaling=1), 4, 1)])
def test_virtual_ranks_w_cycle_and_scaling(lib_built, kw, P, rep):
    """The W-cycle (second coarse visit: halo + coarse residual, the whole
    coarse cycle again, x += e), coarse-grid correction scaling (halo,
    q = A_c e on the owned rows, dot partials all-reduced, alpha on every rank,
    ghosts scaled with their owners) and more than one sweep per smoothing on
    P virtual ranks equal the single-rank oracle apply (src/amg_parameters.py:
    69, 74-75, 78); rep_nodes 1 keeps every level above the coarsest
    distributed."""
    import torch
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(3, 16, 1e6)
    ckw = dict(kw)
    conv = {'smoother': {'POLY': 12}, 'cycle_type': {'W': 2}, 'AMG_type': {'UA': 1}, 'aggregation_type': {'HEM': 5}}
    for k, m in conv.items():
        if k in ckw:
            ckw[k] = m[ckw[k]]
    h = mo.setup(s.scipy(), mo.Params(num_functions=2, **kw), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=rep,
                          num_functions=2, **ckw) for p in range(P)]
    rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
    zs = [torch.zeros_like(x) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, zs)
    torch.cuda.synchronize()
    z = _gather(s, hs, zs)
    assert np.linalg.norm(z - zo) / np.linalg.norm(zo) < 1e-10
    for hh in hs:
        hh.close()


@pytest.mark.parametrize('kw,P,rep', [
    (dict(smoother='SGS', coarse_scaling=1, Schwarz_type=7), 2, 100),
    (dict(smoother='SGS', coarse_scaling=1, Schwarz_type=7), 3, 1),
    (dict(smoother='GS', Schwarz_type=7), 3, 100),
    (dict(smoother='SGS', coarse_scaling=1, Schwarz_type=7, presmooth_iter=2, postsmooth_iter=2), 4, 1),
    (dict(smoother='SGS', coarse_scaling=1, Schwarz_type=7, AMG_type='UA', aggregation_type='HEM',
          cycle_type='W'), 8, 1)])
def test_virtual_ranks_multicolour_gs(lib_built, kw, P, rep):
    """The reference's smoother family on P virtual ranks: multicolour node-
    block GS / SGS (level 0 on the seed blocks) with a halo of each colour's
    nodes after its step, so every colour reads current ghosts -- the same
    sweep as on one GPU (src/amg_parameters.py:72-78).  Equal to the one-GPU
    handle's apply up to summation order, and to the oracle; the last case is
    the reference family (UA + HEM + W-cycle + SGS + coarse scaling) with
    every level above the coarsest distributed."""
    import torch
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(3, 16, 1e6)
    ckw = dict(kw)
    conv = {'smoother': {'SGS': 11, 'GS': 10}, 'cycle_type': {'W': 2}, 'AMG_type': {'UA': 1},
            'aggregation_type': {'HEM': 5}}
    for k, m in conv.items():
        if k in ckw:
            ckw[k] = m[ckw[k]]
    h = mo.setup(s.scipy(), mo.Params(num_functions=2, **kw), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    B1 = M.MetricAMG(s.scipy(), s.W, idofs=s.idofs, num_functions=2, setup='gpu', **ckw)
    z1 = B1 * r
    hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=rep,
                          num_functions=2, **ckw) for p in range(P)]
    rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
    zs = [torch.zeros_like(x) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, zs)
    torch.cuda.synchronize()
    z = _gather(s, hs, zs)
    assert np.linalg.norm(z - z1) / np.linalg.norm(z1) < 1e-12
    assert np.linalg.norm(z - zo) / np.linalg.norm(zo) < 1e-10
    for hh in hs:
        hh.close()
    B1.close()


@pytest.mark.parametrize('case,P,rep', [('bidomain', 3, 100), ('bidomain', 8, 1), ('unfused', 2, 100),
                                         ('emi_poly', 4, 100), ('bidomain2d', 5, 10), ('sell', 3, 100),
                                         ('merged', 2, 100)])
def test_rank_slice_download_bitwise(lib_built, monkeypatch, case, P, rep):
    """The rank-local operators built in HBM from the GPU hierarchy (default;
    ghost lists marked on the device, device.hip dev_rank_ops), from the
    rank's downloaded rows planned on the host, and from the whole
    downloaded hierarchy planned on the host: bitwise equal applies and byte
    counts, also with every level above the coarsest distributed (rep_nodes
    1, 8 ranks), without post fusion, with the seed-split EMI smoother and
    with SELL / [P | AP] storage forced."""
    import torch
    import metric_amg_examples_amd as M
    kw = {}
    if case == 'emi_poly':
        s = M.problems.emi(3, 16, 1e6)
        kw = dict(smoother=12, Schwarz_maxlvl=0)
    elif case == 'bidomain2d':
        s = M.problems.bidomain(2, 64, 1.0)
    else:
        s = M.problems.bidomain(3, 16, 1e6)
    if case == 'unfused':
        kw['post_fusion'] = 0
    elif case == 'sell':
        set_opt('MAMG_SELL_MIN_ROWS', '1')     # SELL / half-symmetric rank-local A with ghosts
    elif case == 'merged':
        set_opt('MAMG_POST_K', '0')
    r = mo.seeded_rhs(s.N)
    out, nbytes = [], []
    for full in ('full', 'rows', ''):   # whole download + host plan, rank rows + host plan, built in HBM
        set_opt('MAMG_DIST_TEST', full)
        hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=rep,
                              num_functions=2, **kw) for p in range(P)]
        rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
        zs = [torch.zeros_like(x) for x in rs]
        M.DistMetricAMG.virtual_apply(hs, rs, zs)
        torch.cuda.synchronize()
        out.append([z.cpu().numpy() for z in zs])
        nbytes.append([hh.apply_bytes for hh in hs])
        for hh in hs:
            hh.close()
    for o in out[1:]:
        for a, b in zip(out[0], o):
            assert np.array_equal(a, b)
    assert nbytes[0] == nbytes[1] == nbytes[2]


@pytest.mark.parametrize('mode', ['unfused', 'sell', 'nohalf', 'merged'])
def test_virtual_ranks_storage_variants(lib_built, monkeypatch, mode):
    """Distributed cycle without post fusion (prolongation, fine halo,
    block-Jacobi sweep), with SELL-64 storage forced onto the rank-local
    operators (K included; the level-0 A then half-symmetric with a ghost
    part), SELL-64 A without the half format, and with the [P | AP] post
    window instead of K = P - W AP: all equal the single-rank oracle apply."""
    import torch
    import metric_amg_examples_amd as M
    kw = {}
    if mode in ('sell', 'nohalf'):
        set_opt('MAMG_SELL_MIN_ROWS', '1')
        set_opt('MAMG_HALF', '1' if mode == 'sell' else '0')
    elif mode == 'merged':
        set_opt('MAMG_POST_K', '0')
    else:
        kw['post_fusion'] = 0
    s = M.problems.bidomain(3, 16, 1e6)
    h = mo.setup(s.scipy(), mo.Params(num_functions=2), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    P = 3
    hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=100,
                          num_functions=2, **kw) for p in range(P)]
    rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
    zs = [torch.zeros_like(x) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, zs)
    torch.cuda.synchronize()
    z = _gather(s, hs, zs)
    assert np.linalg.norm(z - zo) / np.linalg.norm(zo) < 1e-10
    for hh in hs:
        hh.close()


def test_single_rank_rccl(lib_built):
    import torch
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(3, 16, 1e4)
    h = mo.setup(s.scipy(), mo.Params(num_functions=2), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    uid = M.DistMetricAMG.unique_id()
    assert len(uid) == 128
    d = M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=0, nranks=1, comm_id=uid, rep_nodes=100,
                        num_functions=2)
    rt = torch.as_tensor(d.local_slice(r)).cuda()
    zt = torch.zeros_like(rt)
    d.apply_device(rt, zt, torch.cuda.current_stream())
    ms, kms, cb = d.time_apply(rt, zt, 3, 1, torch.cuda.current_stream())
    torch.cuda.synchronize()
    zo = h.apply(r)
    assert np.linalg.norm(zt.cpu().numpy() - zo) / np.linalg.norm(zo) < 1e-10
    assert ms > 0 and d.apply_bytes > 0
    d.close()


def test_single_rank_rccl_graph(lib_built):
    """the distributed apply replayed from a hipGraph with the
    RCCL calls inside the capture (a 1-rank communicator: empty send/receive
    groups, the all-reduces of coarse scaling, the side-stream fork of the
    interior rows) is bitwise the eager apply, replay after replay."""
    import torch
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(3, 16, 1e4)
    r = mo.seeded_rhs(s.N)
    for kw in (dict(), dict(smoother=11, coarse_scaling=1, cycle_type=2, Schwarz_type=7)):
        d = M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=0, nranks=1, comm_id=M.DistMetricAMG.unique_id(),
                            rep_nodes=100, num_functions=2, **kw)
        st = torch.cuda.current_stream()
        rt = torch.as_tensor(d.local_slice(r)).cuda()
        ze, zg = torch.zeros_like(rt), torch.full_like(rt, float('nan'))
        d.apply_device(rt, ze, st)
        d.apply_graph(rt, zg, st)
        torch.cuda.synchronize()
        assert torch.equal(ze, zg)
        zg.fill_(float('nan'))
        ms, _, _ = d.time_apply(rt, zg, 3, 2, st)       # graph replays
        torch.cuda.synchronize()
        assert ms > 0 and torch.equal(ze, zg)
        h = mo.setup(s.scipy(), mo.Params(num_functions=2, **({} if not kw else dict(
            smoother='SGS', coarse_scaling=1, cycle_type='W', Schwarz_type=7))), idofs=s.idofs)
        zo = h.apply(r)
        assert np.linalg.norm(ze.cpu().numpy() - zo) / np.linalg.norm(zo) < 1e-10
        d.close()


@pytest.mark.parametrize('P,kw', [(2, {}), (3, dict(smoother=11, coarse_scaling=1, cycle_type=2, Schwarz_type=7)),
                                  (8, dict(smoother=12))])
def test_virtual_ranks_graph_bitwise(lib_built, monkeypatch, P, kw):
    """The virtual ranks' lockstep apply captured into one hipGraph (every
    rank's kernels, halo packs, device-copy exchanges, reverse-adds and
    all-reduce sums) is bitwise the eager lockstep apply: Jacobi (the
    overlap split of the half-symmetric A), SGS + scaling + W (colour halos,
    all-reduces), POLY at P = 8."""
    import torch
    import metric_amg_examples_amd as M
    set_opt('MAMG_SELL_MIN_ROWS', '1')
    s = M.problems.bidomain(3, 16, 1e6)
    r = mo.seeded_rhs(s.N)
    hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=100,
                          num_functions=2, **kw) for p in range(P)]
    rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
    ze = [torch.zeros_like(x) for x in rs]
    zg = [torch.full_like(x, float('nan')) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, ze)
    M.DistMetricAMG.virtual_apply(hs, rs, zg, graph=True)
    torch.cuda.synchronize()
    for a, b in zip(ze, zg):
        assert torch.equal(a, b)
    for hh in hs:
        with pytest.raises(M._lib.MamgError):      # no communicator: the graph path is refused
            hh.apply_graph(rs[0], zg[0])
        hh.close()


@pytest.mark.parametrize('preset,P', [('schwarz', 2), ('schwarz', 3), ('patch', 4), ('patch', 8)])
def test_virtual_ranks_node_patches(lib_built, preset, P):
    """the reference's level-0 smoother on N ranks.  The
    preset the north-star driver passes (parameters_metric_schwarz, src/
    bidomain_3d.py:144-147: UA + HEM + W + SGS + scaling + SCHWARZ_SYMMETRIC
    1-rings = the node patches) and the GPU profile with the patches
    (parameters_metric_mi355x_patch), row-partitioned over P virtual ranks:
    every rank colours the whole level-0 graph (the same colours), computes
    the patches centred within 1 hop of its nodes, and after each colour
    exchanges the nodes that colour's patches wrote within 3 hops.  The
    gathered apply equals the one-GPU apply to 1e-12 and the oracle's to
    1e-10; the lockstep graph replay equals the eager run bitwise."""
    import torch
    import metric_amg_examples_amd as M
    Pm = M.parameters
    params = Pm.parameters_metric_schwarz if preset == 'schwarz' else Pm.parameters_metric_mi355x_patch
    s = M.problems.bidomain(3, 16, 1e6)
    r = mo.seeded_rhs(s.N)
    B1 = M.MetricAMG(s, s.W, idofs=s.idofs, parameters=params)
    assert B1.level_format(0)['patches']
    z1 = B1 * r
    hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, parameters=params, rank=p, nranks=P, comm_id=None,
                          rep_nodes=100) for p in range(P)]
    rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
    zs = [torch.zeros_like(x) for x in rs]
    zg = [torch.full_like(x, float('nan')) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, zs)
    M.DistMetricAMG.virtual_apply(hs, rs, zg, graph=True)
    torch.cuda.synchronize()
    z = _gather(s, hs, zs)
    assert np.linalg.norm(z - z1) / np.linalg.norm(z1) < 1e-12
    for a, b in zip(zs, zg):
        assert torch.equal(a, b)
    if preset == 'schwarz':
        from test_gpu_patch import _oracle_params
        h = mo.setup(s.scipy(), _oracle_params(params, num_functions=2), idofs=s.idofs)
        zo = h.apply(r)
        assert np.linalg.norm(z - zo) / np.linalg.norm(zo) < 1e-10
    for hh in hs:
        hh.close()
    B1.close()


@pytest.mark.parametrize('P', [2, 4])
def test_virtual_ranks_half_bitwise(lib_built, monkeypatch, P):
    """Rank-local level-0 A in the half-symmetric format (owned part through
    mirrors, ghost columns in their own part) sums each row in its local
    column order: bitwise the SELL-64 result, with fewer bytes per apply."""
    import torch
    import metric_amg_examples_amd as M
    set_opt('MAMG_SELL_MIN_ROWS', '1')
    s = M.problems.bidomain(3, 16, 1e6)
    r = mo.seeded_rhs(s.N)
    out, nbytes = [], []
    for half in ('1', '0'):
        set_opt('MAMG_HALF', half)
        hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=100,
                              num_functions=2) for p in range(P)]
        rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
        zs = [torch.zeros_like(x) for x in rs]
        M.DistMetricAMG.virtual_apply(hs, rs, zs)
        torch.cuda.synchronize()
        out.append([z.cpu().numpy() for z in zs])
        nbytes.append(sum(hh.apply_bytes for hh in hs))
        for hh in hs:
            hh.close()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)
    assert nbytes[0] < nbytes[1]


@pytest.mark.parametrize('P', [1, 3])
def test_dist_pcg_virtual_ranks(lib_built, P):
    """DistConjGrad on P virtual ranks (rank-local SpMV with halo, distributed
    V-cycle, dots summed over ranks): iteration count and residual history of
    the oracle PCG; the rank SpMV equals the global SpMV's rows."""
    import torch
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(3, 16, 1e4)
    A = s.scipy()
    h = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs)
    b = mo.seeded_rhs(s.N)
    ref = mo.pcg(A, h.apply, b, 1e-8, 500)
    hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=100,
                          num_functions=2) for p in range(P)]
    xs = [torch.as_tensor(hh.local_slice(b)).cuda() for hh in hs]
    ys = [torch.zeros_like(x) for x in xs]
    if P > 1:
        M.DistMetricAMG.virtual_spmv(hs, xs, ys)
    else:
        hs[0].spmv_device(xs[0], ys[0])
    torch.cuda.synchronize()
    yo = A @ b
    for hh, y in zip(hs, ys):
        assert np.allclose(y.cpu().numpy(), hh.local_slice(yo), rtol=1e-13, atol=1e-13 * np.abs(yo).max())
    cg = M.DistConjGrad.for_handles(hs if P > 1 else hs[0], tolerance=1e-8, maxiter=500)
    x = _gather(s, hs, cg.solve([torch.as_tensor(hh.local_slice(b)).cuda() for hh in hs]))
    assert len(cg.residuals) == len(ref.residuals)
    assert np.allclose(cg.residuals, ref.residuals, rtol=1e-6, atol=0)
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) < 1e-6
    for hh in hs:
        hh.close()


@pytest.mark.parametrize('n,P,sell', [(16, 3, '1'), (32, 2, '1'), (32, 3, str(1 << 20))])
def test_virtual_ranks_overlap_bitwise(lib_built, monkeypatch, n, P, sell):
    """Residual split into the ghost-free row window (run while the halo is
    in flight) and the boundary rows (after it), and level 0's K split the
    same way around the coarse-e halo (its rows without coarse ghost columns
    in 256-row runs, SELL K or the lane-group BSR K): bitwise the unsplit
    apply, for the cycle and the rank SpMV."""
    import torch
    import metric_amg_examples_amd as M
    set_opt('MAMG_SELL_MIN_ROWS', sell)
    s = M.problems.bidomain(3, n, 1e6)
    r = mo.seeded_rhs(s.N)
    out = []
    forks = []
    for ov in ('1', '0'):
        set_opt('MAMG_OVERLAP', ov)
        hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=100,
                              num_functions=2) for p in range(P)]
        rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
        zs = [torch.zeros_like(x) for x in rs]
        ys = [torch.zeros_like(x) for x in rs]
        M.DistMetricAMG.virtual_apply(hs, rs, zs)
        M.DistMetricAMG.virtual_spmv(hs, rs, ys)
        torch.cuda.synchronize()
        out.append([z.cpu().numpy() for z in zs] + [y.cpu().numpy() for y in ys])
        forks.append([hh.apply_launches['stream_forks'] for hh in hs])
        for hh in hs:
            hh.close()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)
    assert all(f == 0 for f in forks[1])
    print('stream forks per apply with the overlap', forks[0])
    # K's split always; the residual's window with the half-symmetric A (SELL sizes)
    assert all(f >= (2 if sell == '1' else 1) for f in forks[0])


def test_virtual_ranks_band_schedule_bitwise(lib_built, monkeypatch):
    """Band schedule on the rank-local half-symmetric A (full-range launch
    and the ghost-free interior run launched during the halo) at 3-D n=128 on
    2 ranks, where it engages: cycle and rank SpMV bitwise equal to row
    order."""
    import torch
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(3, 128, 1e6)
    r = mo.seeded_rhs(s.N)
    P = 2
    out = []
    for bands in ('1', '0'):
        set_opt('MAMG_HALF_BANDS', bands)
        hs = [M.DistMetricAMG(s, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None,
                              num_functions=2) for p in range(P)]
        rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
        zs = [torch.zeros_like(x) for x in rs]
        ys = [torch.zeros_like(x) for x in rs]
        M.DistMetricAMG.virtual_apply(hs, rs, zs)
        M.DistMetricAMG.virtual_spmv(hs, rs, ys)
        torch.cuda.synchronize()
        out.append([z.cpu().numpy() for z in zs] + [y.cpu().numpy() for y in ys])
        for hh in hs:
            hh.close()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _host_exchange_worker(rank, world, port, q, problem, kw):
    """one rank process: the product's rank-local handle on the (shared) GPU,
    its exchanges through the host-staged gloo transport"""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, 'oracle')):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import metric_amg_examples_amd as M
        import mamg_oracle
        s = M.problems.emi(3, 16, 1e6) if problem == 'emi' else M.problems.bidomain(3, 16, 1e6)
        A = s.tocsr() if problem == 'emi' else s
        h = M.DistMetricAMG(A, s.W, idofs=s.idofs, rank=rank, nranks=world, comm_id=None, rep_nodes=100,
                            exchange='gloo', num_functions=2, **kw)
        r = torch.as_tensor(h.local_slice(mamg_oracle.seeded_rhs(s.N))).cuda()
        z = torch.zeros_like(r)
        h.apply_device(r, z)
        torch.cuda.synchronize()
        cg = M.DistConjGrad.for_handles(h, tolerance=1e-8, maxiter=500)
        x = cg.solve([r.clone()])[0]
        torch.cuda.synchronize()
        q.put((rank, h.o0, h.o1, z.cpu().numpy(), x.cpu().numpy(), list(cg.residuals), h.apply_launches))
        h.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('problem,kw', [('bidomain', {}), ('emi', dict(smoother=12, Schwarz_maxlvl=0)),
                                        ('bidomain', dict(smoother=11, coarse_scaling=1, Schwarz_type=7)),
                                        ('bidomain', dict(Schwarz_type=6))])
def test_two_processes_host_exchange(lib_built, problem, kw):
    """Two rank processes on the one GPU of the box, exchanging through the
    host-staged gloo transport (RCCL refuses two ranks on one GPU): each
    builds its plan and rank-local operators in its own process and runs the
    product's pack / halo / reverse-add / all-reduce schedule; the gathered
    apply equals the oracle's, and DistConjGrad (dots all-reduced over gloo)
    has the oracle PCG's iteration count and residuals."""
    import torch.multiprocessing as mp
    import metric_amg_examples_amd as M
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_exchange_worker, args=(r, 2, port, q, problem, kw)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s = M.problems.emi(3, 16, 1e6) if problem == 'emi' else M.problems.bidomain(3, 16, 1e6)
    okw = {}
    if kw.get('smoother') == 12:
        okw = {'smoother': 'POLY', 'Schwarz_maxlvl': 0}
    elif kw.get('smoother') == 11:
        okw = {'smoother': 'SGS', 'coarse_scaling': 1, 'Schwarz_type': 7}
    elif kw.get('Schwarz_type') == 6:       # node patches (colour halos through the host-staged transport)
        okw = {'Schwarz_type': 6}
    A = s.scipy()
    h = mo.setup(A, mo.Params(num_functions=2, **okw), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    ref = mo.pcg(A, h, r, 1e-8, 500)
    z, x = np.zeros(s.N), np.zeros(s.N)
    for rank, o0, o1, zl, xl, resid, launches in res:
        # what one apply issues per rank: printed for DESIGN
        print('rank', rank, problem, kw, launches)
        assert launches['kernels'] > 10 and launches['p2p_groups'] > 0 and launches['p2p_messages'] > 0
        nloc = o1 - o0
        z[o0:o1], z[s.nv + o0:s.nv + o1] = zl[:nloc], zl[nloc:]
        x[o0:o1], x[s.nv + o0:s.nv + o1] = xl[:nloc], xl[nloc:]
        assert len(resid) == len(ref.residuals)
        assert np.allclose(resid, ref.residuals, rtol=1e-6, atol=0)
    assert np.linalg.norm(z - zo) / np.linalg.norm(zo) < 1e-10
    assert np.linalg.norm(x - ref.x) / np.linalg.norm(ref.x) < 1e-6


@pytest.mark.parametrize('dim,n', [(2, 64), (3, 16), (3, 33)])
def test_device_generator_bitwise(lib_built, dim, n):
    """mamg_gen_bidomain_device (gfx950 kernels, no FMA contraction) builds
    the host generator's matrix bit for bit."""
    import metric_amg_examples_amd as M
    s = M.problems.bidomain(dim, n, 1e6)
    ip, ix, dv = M.problems.bidomain_device(dim, n, 1e6)
    assert np.array_equal(ip.cpu().numpy(), s.indptr)
    assert np.array_equal(ix.cpu().numpy(), s.indices)
    assert np.array_equal(dv.cpu().numpy(), s.data)


@pytest.mark.parametrize('P,kw', [(2, {}), (4, dict(smoother='SGS', coarse_scaling=1, cycle_type='W'))])
def test_dist_setup_from_device_matrix(lib_built, P, kw):
    """mamg_setup_dist_device: every rank sets up from A_0 generated in its
    HBM (no host matrix); the virtual-rank applies are bitwise those of the
    ranks set up from the host matrix, and equal the oracle."""
    import torch
    import metric_amg_examples_amd as M
    ck = dict(kw)
    if 'smoother' in ck:
        ck['smoother'] = {'SGS': 11}[ck['smoother']]
        ck['Schwarz_type'] = M.parameters.SCHWARZ_SEED_BLOCKS
    if 'cycle_type' in ck:
        ck['cycle_type'] = {'W': 2}[ck['cycle_type']]
    s = M.problems.bidomain(3, 16, 1e6)
    A0 = M.problems.bidomain_device(3, 16, 1e6)
    meta = M.problems.bidomain_meta(3, 16, int(A0[1].numel()))
    r = mo.seeded_rhs(s.N)
    outs = []
    for A in (s, A0):
        hs = [M.DistMetricAMG(A, meta.W, idofs=meta.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=100,
                              num_functions=2, **ck) for p in range(P)]
        rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
        zs = [torch.zeros_like(x) for x in rs]
        M.DistMetricAMG.virtual_apply(hs, rs, zs)
        torch.cuda.synchronize()
        outs.append(_gather(s, hs, zs))
        for hh in hs:
            hh.close()
    assert np.array_equal(outs[0], outs[1])
    okw = dict(kw, Schwarz_type=7) if kw else {}
    h = mo.setup(s.scipy(), mo.Params(num_functions=2, **okw), idofs=s.idofs)
    assert np.linalg.norm(outs[0] - h.apply(r)) / np.linalg.norm(outs[0]) < 1e-10
