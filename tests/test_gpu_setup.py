"""GPU setup (mamg_setup_gpu, csrc/gsetup.hip) against the host setup.

Contract: for the nodal 2-field profile the GPU
builds the SAME hierarchy as the C++ host setup, bit for bit -- node graph,
strength, MIS-2 aggregates, smoother blocks, SA prolongator, R = P^T,
Galerkin coarse operators, coarsest inverse -- and the host setup is itself
bitwise equal to the oracle (tests/test_host_setup.py, tests/test_golden.py).
So: every exported level array is np.array_equal, and an apply through a
GPU-setup handle equals the host-setup handle's apply exactly (same device
kernels on identical bits), hence the oracle's to 1e-10.
"""
import numpy as np
import pytest

import mamg_oracle as mo
from conftest import set_opt

pytestmark = pytest.mark.gpu


def _mamg():
    import metric_amg_examples_amd as M
    return M


CASES = [
    (2, 32, 1.0, dict()),
    (2, 64, 1e6, dict()),
    (3, 8, 1e6, dict()),
    (3, 16, 1e4, dict()),
    (3, 16, 1e10, dict()),
    (3, 16, 1e2, dict(strong_coupled=0.08)),
    (2, 32, 1e3, dict(AMG_type=1)),                 # UA: P = T
    (3, 16, 1e6, dict(post_fusion=0)),
    (2, 32, 1e3, dict(Schwarz_mmsize=1)),           # level-0 seed blocks split into singletons
    (2, 64, 1e4, dict(coarse_dof=400, max_levels=3)),
    # parallel heavy-edge matching (aggregation_type HEM), UA and SA
    (3, 16, 1e6, dict(aggregation_type=5, AMG_type=1)),
    (2, 64, 1e2, dict(aggregation_type=5)),
    (3, 16, 1e10, dict(aggregation_type=5, AMG_type=1)),
    # sequential Vanek-Mandel-Brezina (aggregation_type VMB): the GPU setup
    # runs this one step on the host, on the strong graph it built
    (3, 16, 1e6, dict(aggregation_type=1, AMG_type=1, strong_coupled=0.1)),
    (2, 64, 1e4, dict(aggregation_type=1)),
]


def hierarchies_equal(Hh, Hg):
    assert Hh.num_levels == Hg.num_levels
    for l in range(Hh.num_levels):
        a, b = Hh.level(l, with_A=(l > 0)), Hg.level(l, with_A=(l > 0))
        assert a.keys() == b.keys(), (l, a.keys(), b.keys())
        for k in a:
            if k == 'n':
                assert a[k] == b[k]
                continue
            x, y = a[k], b[k]
            if isinstance(x, tuple):
                for u, v in zip(x[:3], y[:3]):
                    assert np.array_equal(u, v), (l, k)
                assert x[3] == y[3]
            else:
                assert np.array_equal(x, y), (l, k)


@pytest.mark.parametrize('dim,n,g,kw', CASES)
def test_gpu_hierarchy_bitwise_equals_host(lib_built, dim, n, g, kw):
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    Hh = M.HostHierarchy(s, idofs=s.idofs, num_functions=2, **kw)
    Hg = M.HostHierarchy(s, idofs=s.idofs, num_functions=2, gpu=True, **kw)
    hierarchies_equal(Hh, Hg)
    Hh.close()
    Hg.close()


@pytest.mark.parametrize('stage', [('16', '16', '1'), ('16', '128', '1'), ('16', '128', '0'), ('0', '128', '1')])
@pytest.mark.parametrize('dim,n,g,kw', [(3, 16, 1e6, dict()), (2, 64, 1e4, dict(aggregation_type=5)),
                                        (3, 16, 1e6, dict(AMG_type=1))])
def test_gpu_spgemm_staging_bitwise(lib_built, monkeypatch, dim, n, g, kw, stage):
    """The one-pass SpGEMM (count pass staging rows of <= stride entries,
    compacted after the scan; longer rows through the fill launch), with
    the node's two rows of the 2-function matrices taken together
    (spgemm_pair_kernel) or row by row: stride 16 (most Galerkin rows take
    the long-row list), the default stride, pairs off, and staging off all
    give the host setup's hierarchy bit for bit."""
    M = _mamg()
    gb, stride, pair = stage
    set_opt('MAMG_SPGEMM_STAGE_GB', gb)
    set_opt('MAMG_SPGEMM_STAGE_STRIDE', stride)
    set_opt('MAMG_SPGEMM_PAIR', pair)
    s = M.problems.bidomain(dim, n, g)
    Hh = M.HostHierarchy(s, idofs=s.idofs, num_functions=2, **kw)
    Hg = M.HostHierarchy(s, idofs=s.idofs, num_functions=2, gpu=True, **kw)
    hierarchies_equal(Hh, Hg)
    Hh.close()
    Hg.close()


@pytest.mark.parametrize('knob', ['MAMG_CSR2BSR_FILL', 'MAMG_MIS_STAGED'])
@pytest.mark.parametrize('dim,n,g,kw', [(3, 16, 1e6, dict()), (2, 64, 1e4, dict(post_fusion=0)),
                                        (3, 32, 1e6, dict(smoother=12)), (3, 16, 1e2, dict(AMG_type=1))])
def test_csr2bsr_fill_variants_bitwise(lib_built, monkeypatch, dim, n, g, kw, knob):
    """The device CSR -> BSR2 fill pass with columns only in LDS (slots
    written in place, values scattered by a coalesced sweep; default) and the
    column + value staged merge (MAMG_CSR2BSR_FILL=0) give the same layouts:
    every level's format and the applies are equal bit for bit.  Likewise the
    MIS-2 maxima over staged rows and the lane-per-row walks
    (MAMG_MIS_STAGED=0)."""
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    outs, fmts = [], []
    for f in ('1', '0'):
        set_opt(knob, f)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **kw)
        fmts.append([B.level_format(lv) for lv in range(B.num_levels)])
        outs.append([B * mo.seeded_rhs(s.N, seed) for seed in (1234, 7)])
        B.close()
    assert fmts[0] == fmts[1]
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize('nranks', [2, 3, 8])
@pytest.mark.parametrize('dim,n,g,kw', [(3, 16, 1e6, dict()), (2, 64, 1e4, dict()), (3, 16, 1e6, dict(AMG_type=1)),
                                        (3, 24, 1e2, dict(aggregation_type=5))])
def test_sharded_galerkin_equals_hierarchy(lib_built, dim, n, g, kw, nranks):
    """The start of a partition-local setup: the Galerkin
    products row-sharded over virtual ranks -- each rank's (A P) rows from its
    A rows and the P rows of its halo, its coarse rows from its R rows and the
    (A P) rows of the fine dofs they reach, taken from their owners' sharded
    results -- equal the GPU hierarchy's next level bit for bit, at levels 0
    and 1, and the halos are really read."""
    import ctypes as C
    M = _mamg()
    L = M._lib
    s = M.problems.bidomain(dim, n, g)
    H = M.HostHierarchy(s, idofs=s.idofs, num_functions=2, gpu=True, **kw)
    A0 = s.scipy().tocsr()
    A0.sort_indices()
    for lv in range(min(2, H.num_levels - 1)):
        cur = H.level(lv, with_A=lv > 0)
        nxt = H.level(lv + 1, with_A=True)
        A = cur['A'] if lv > 0 else (A0.indptr.astype(np.int64), A0.indices.astype(np.int32),
                                     A0.data.astype(np.float64), A0.shape)
        mats = [A, cur['P'], nxt['A']]
        st = [L.as_csr_struct(np.ascontiguousarray(m[0], np.int64), np.ascontiguousarray(m[1], np.int32),
                              np.ascontiguousarray(m[2], np.float64), m[3][1]) for m in mats]
        res = np.zeros(6, np.int64)
        L.check(L.lib().mamg_sharded_galerkin_check(C.byref(st[0]), C.byref(st[1]), C.byref(st[2]), nranks, 0,
                                                    L.ptr(res, C.c_int64)))
        print('level', lv, 'ranks', nranks, 'res', res.tolist())
        assert res[0] == 0 and res[1] == 0, res
        assert res[4] == A[3][0] and res[5] == nxt['A'][3][0]
        assert res[2] > 0 and res[3] > 0


@pytest.mark.parametrize('dim,n,g,kw', CASES)
def test_gpu_setup_apply_bitwise_equals_host_setup(lib_built, dim, n, g, kw):
    M = _mamg()
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    Bg = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup='gpu', **kw)
    Bh = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup='host', **kw)
    assert Bg.setup_path == 'gpu' and Bh.setup_path == 'host'
    assert Bg.num_levels == Bh.num_levels
    for lv in range(Bg.num_levels):
        assert Bg.level_format(lv) == Bh.level_format(lv)
    for seed in (1234, 7):
        r = mo.seeded_rhs(s.N, seed)
        assert np.array_equal(Bg * r, Bh * r)
    oracle_kw = {k: v for k, v in kw.items() if k != 'post_fusion'}
    if 'AMG_type' in oracle_kw:
        oracle_kw['AMG_type'] = {1: 'UA', 2: 'SA'}[oracle_kw['AMG_type']]
    if 'aggregation_type' in oracle_kw:
        oracle_kw['aggregation_type'] = {1: 'VMB', 2: 'MIS', 5: 'HEM'}[oracle_kw['aggregation_type']]
    h = mo.setup(A, mo.Params(num_functions=2, **oracle_kw), idofs=s.idofs)
    r = mo.seeded_rhs(s.N)
    zo = h.apply(r)
    tol = 1e-10 if g < 1e8 else 1e-8
    assert np.linalg.norm(Bg * r - zo) / np.linalg.norm(zo) < tol
    t = Bg.setup_timings
    assert t['setup_total'] > 0 and t['layout'] > 0


def test_gpu_setup_device_input_and_pcg(lib_built):
    """A handed over in HBM (torch tensors): same handle bits; PCG through it
    takes the oracle's iteration count."""
    import torch
    M = _mamg()
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    dA = (torch.as_tensor(s.indptr).cuda(), torch.as_tensor(s.indices).cuda(),
          torch.as_tensor(s.data).cuda())
    Bd = M.MetricAMG(dA, s.W, idofs=s.idofs, num_functions=2)
    Bh = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup='host')
    r = mo.seeded_rhs(s.N)
    assert np.array_equal(Bd * r, Bh * r)
    Bd._Aop = A
    solver = M.ConjGrad(A, precond=Bd, tolerance=1e-8, maxiter=500)
    solver * r
    ref = mo.pcg(A, mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs), r, 1e-8, 500)
    assert len(solver.residuals) == len(ref.residuals)


def _generic_case(name):
    """(A, W, idofs, parameter overrides) of the hierarchies whose smoothers
    are not 2x2 node blocks: general seed blocks, overlapping seed rings
    (SCHWARZ_ADDITIVE), point smoothers, scalar (num_functions 1) AMG."""
    M = _mamg()
    P = M.parameters
    if name.startswith('emi'):            # EMI interface seeds: not node-aligned
        s = M.problems.emi(3, 16, 1e6)
        kw = dict(num_functions=2)
        if name == 'emi_rings2':          # the reference's EMI default: 2-rings (src/utils.py:78)
            kw.update(Schwarz_type=P.SCHWARZ_ADDITIVE, Schwarz_maxlvl=2)
        if name == 'emi_rings2_poly':
            kw.update(Schwarz_type=P.SCHWARZ_ADDITIVE, Schwarz_maxlvl=2, smoother=P.SMOOTHER_POLY)
        return s.tocsr(), s.W, s.idofs, kw
    if name.startswith('3d1d'):           # BASELINE config 5: scalar, additive 2-rings
        s = M.problems.emi_3d1d(16, 1e4, 1.0 if name.endswith('r1') else 0.0)
        return s.scipy(), s.W, s.idofs, dict(parameters=P.parameters_metric_3d1d)
    s = M.problems.bidomain(3, 16, 1e4)
    A = s.scipy()
    if name == 'every3rd':                # seeds that do not pair up by node
        return A, s.W, np.arange(0, s.N, 3, dtype=np.int32), dict(num_functions=2)
    if name == 'nodal_point_smoother':    # node aggregates, point Jacobi, nodal SA
        return A, s.W, None, dict(num_functions=2, node_block_smoother=0)
    if name == 'nodal_point_sa':          # node aggregates, point SA prolongator
        return A, s.W, None, dict(num_functions=2, sa_block_diag=0)
    scalar = dict(num_functions=1)        # plain AMG (src/utils.py:15-42)
    extra = {'scalar': {}, 'scalar_rho_iters': dict(rho_iters=5), 'scalar_ua': dict(AMG_type=1),
             'scalar_hem': dict(aggregation_type=5), 'scalar_l1': dict(smoother=P.SMOOTHER_L1DIAG),
             'scalar_jacobi': dict(smoother=P.SMOOTHER_JACOBI, strong_coupled=0.08),
             'scalar_poly': dict(smoother=P.SMOOTHER_POLY)}[name]
    return A, None, None, dict(scalar, **extra)


GENERIC = ['emi_blocks', 'emi_rings2', 'emi_rings2_poly', '3d1d_r0', '3d1d_r1', 'every3rd',
           'nodal_point_smoother', 'nodal_point_sa', 'scalar', 'scalar_rho_iters', 'scalar_ua',
           'scalar_hem', 'scalar_l1', 'scalar_jacobi', 'scalar_poly']


@pytest.mark.parametrize('name', GENERIC)
def test_gpu_setup_generic_smoothers_bitwise(lib_built, name):
    """The GPU setup of hierarchies without 2x2 node-block smoothers (general
    seed blocks, SCHWARZ_ADDITIVE rings, point smoothers, scalar AMG) equals
    the host setup bit for bit, level by level, and its CSR-layout handle
    applies bitwise like the host setup's."""
    M = _mamg()
    A, W, idofs, kw = _generic_case(name)
    Hh = M.HostHierarchy(A, idofs=idofs, **kw)
    Hg = M.HostHierarchy(A, idofs=idofs, gpu=True, **kw)
    hierarchies_equal(Hh, Hg)
    Hh.close()
    Hg.close()
    Bg = M.MetricAMG(A, W, idofs=idofs, setup='gpu', **kw)
    Bh = M.MetricAMG(A, W, idofs=idofs, setup='host', **kw)
    # node-block smoothers with a point SA prolongator keep the BSR2 layout
    assert Bg.setup_path == 'gpu' and Bg.layout == Bh.layout == ('bsr2' if name == 'nodal_point_sa' else 'csr')
    assert Bg.num_levels == Bh.num_levels
    for seed in (1234, 7):
        r = mo.seeded_rhs(A.shape[0], seed)
        assert np.array_equal(Bg * r, Bh * r)
    auto = M.MetricAMG(A, W, idofs=idofs, **kw)      # 'auto' takes the GPU setup now
    assert auto.setup_path == 'gpu'


def test_gpu_setup_rejects_unsupported_and_bad_input(lib_built):
    M = _mamg()
    s = M.problems.bidomain(2, 16, 1e3)
    A = s.scipy()
    # multicolour GS needs node-block smoothers: refused with the host's message
    idofs = np.arange(0, s.N, 3, dtype=np.int32)
    with pytest.raises(M._lib.MamgError) as ei:
        M.MetricAMG(A, s.W, idofs=idofs, num_functions=2, smoother=M.parameters.SMOOTHER_SGS,
                    Schwarz_type=M.parameters.SCHWARZ_SEED_BLOCKS, setup='gpu')
    assert ei.value.code == -4 and 'BSR2' in str(ei.value)
    with pytest.raises(M._lib.MamgError) as ei:           # three fields
        M.MetricAMG(A[:3 * (s.N // 3), :3 * (s.N // 3)].tocsr(), num_functions=3, setup='gpu')
    assert ei.value.code == -4
    # unsorted columns in a row
    ip, ix, dv = s.indptr.copy(), s.indices.copy(), s.data.copy()
    ix[ip[5]], ix[ip[5] + 1] = ix[ip[5] + 1], ix[ip[5]]
    with pytest.raises(M._lib.MamgError) as ei:
        M.MetricAMG((ip, ix, dv), s.W, idofs=s.idofs, num_functions=2, setup='gpu')
    assert ei.value.code == -1


def test_gpu_setup_large_3d_bitwise(lib_built):
    """bidomain_3d n=64 (N = 550k): the whole hierarchy bitwise equal."""
    M = _mamg()
    s = M.problems.bidomain(3, 64, 1e6)
    Hh = M.HostHierarchy(s, idofs=s.idofs, num_functions=2)
    Hg = M.HostHierarchy(s, idofs=s.idofs, num_functions=2, gpu=True)
    hierarchies_equal(Hh, Hg)


def test_setups_with_kept_cache_then_released_bitwise(lib_built):
    """The GPU setups keep their temporaries' blocks cached for the process's
    next setup (capi.cpp TmpTrim, MAMG_TMP_KEEP): a setup from reused blocks,
    and one after mamg_release_setup_cache, give the same applies bit for bit."""
    M = _mamg()
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    outs = []
    for k in range(3):
        if k == 2:
            M.release_setup_cache()
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        outs.append(B * mo.seeded_rhs(s.N, 1234))
        B.close()
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])


def test_setup_cache_limit_bounds_idle_blocks(lib_built):
    """mamg_set_setup_cache_limit: the default bound is
    an eighth of the device's HBM and a setup leaves at most that much idle
    (the SpGEMM staging block included); limit 0 leaves nothing; the applies
    are the same bits either way."""
    import ctypes as C
    import torch
    M = _mamg()
    L = M._lib.lib()
    s = M.problems.bidomain(3, 16, 1e6)
    A = s.scipy()
    idle, lim = C.c_int64(), C.c_int64()
    outs = []
    try:
        for limit in (-1, 0, 1 << 20):
            M._lib.check(L.mamg_set_setup_cache_limit(limit))
            B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
            M._lib.check(L.mamg_setup_cache_bytes(torch.cuda.current_device(), C.byref(idle), C.byref(lim)))
            if limit < 0:
                assert lim.value == torch.cuda.get_device_properties(0).total_memory // 8
            else:
                assert lim.value == limit
            assert 0 <= idle.value <= lim.value, (limit, idle.value, lim.value)
            outs.append(B * mo.seeded_rhs(s.N, 1234))
            B.close()
    finally:
        L.mamg_set_setup_cache_limit(-1)
    assert all(np.array_equal(outs[0], o) for o in outs[1:])


def test_concurrent_setups_share_the_staging_block_safely(lib_built):
    """host threads setting up and applying on one device at
    once.  Single-GPU setups take the library's capture lock (the HIP runtime
    invalidates a stream capture when another thread issues legacy
    null-stream work, so setups never overlap a capture and run one at a
    time); the SpGEMM staging block is leased per product; every thread's
    apply equals a lone setup's bit for bit."""
    import threading
    M = _mamg()
    s = M.problems.bidomain(3, 24, 1e6)
    A = s.scipy()
    r = mo.seeded_rhs(s.N, 1234)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
    ref = B * r
    B.close()
    outs, errs = [None] * 4, []

    def run(k):
        try:
            h = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
            outs[k] = h * r
            h.close()
        except Exception as e:          # noqa: BLE001 -- reported below
            errs.append(repr(e))
    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for o in outs:
        assert np.array_equal(o, ref)
