"""Every BASELINE.json configuration on the GPU, at its full size (VERDICT r1
items N1 / 'untested configs'):

* bidomain_2d nrefs=6 gamma=1e6 (2-D n=1024, N=2.1M) and bidomain_3d nrefs=6
  gamma=1e6 (3-D n=256, N=34M, the north-star config): one GPU apply against
  the oracle's C cycle (oracle/vcycle_ref.c) on the same hierarchy (the GPU
  setup's, copied back; the setup is bitwise the oracle's, tests/
  test_gpu_setup.py) to 1e-10, and the PCG iteration count of the device PCG
  equal to the CPU PCG's (oracle_pcg: the C cycle + C SpMV, cbc.block
  ConjGrad, tolerance 1e-8 absolute, src/bidomain_3d.py:149-157), residual
  histories within 1e-6.
* bidomain_3d nrefs=5 (N=4.3M): the same.
* emi_3d nrefs=5 gamma=1e6 (n=64, N=278,850; src/emi_3d.py:119-143, tolerance
  1e-10): block-form preconditioner R^T Minv R, device apply and PCG against
  the C cycle on the host-setup hierarchy (CSR layout).
The bench's own line repeats the 3-D nrefs=6 PCG check (pcg.cpu_pcg).
"""
import sys
import time

import numpy as np
import pytest

import mamg_oracle as mo

pytestmark = pytest.mark.gpu


def _M():
    import metric_amg_examples_amd as M
    return M


def say(*a):
    print('[configs]', *a, file=sys.stderr, flush=True)


def rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def c_hierarchy(H, sysm_or_A):
    import cref
    M = _M()
    ip, ix, dv, n, _ = M.amg.csr_arrays(sysm_or_A)
    lv = [H.level(l, with_A=(l > 0)) for l in range(H.num_levels)]
    lv[0]['A'] = (ip, ix, dv, (n, n))
    p = H.params
    return cref.CHierarchy(lv, p.cycle_type == 2, p.presmooth_iter, p.postsmooth_iter, p.maxit)


@pytest.mark.parametrize('dim,nrefs', [(2, 6), (3, 5), (3, 6)])
def test_bidomain_baseline_config_apply_and_pcg(lib_built, dim, nrefs):
    import torch
    M = _M()
    n = M.problems.finest_n(dim, nrefs)
    t0 = time.time()
    s = M.problems.bidomain(dim, n, 1e6)
    say('%dD n=%d N=%d generated in %.1fs' % (dim, n, s.N, time.time() - t0))
    B = M.MetricAMG(s, s.W, idofs=s.idofs, num_functions=2, setup='gpu')
    r = M.problems.seeded_rhs(s.N)
    rt = torch.as_tensor(r).cuda()
    z = B.matvec(rt).cpu().numpy()
    H = M.HostHierarchy(s, idofs=s.idofs, num_functions=2, gpu=True)
    assert H.num_levels == B.num_levels
    ch = c_hierarchy(H, s)
    zc = ch.apply(r)
    say('apply rel diff GPU vs C cycle: %.2e' % rel(z, zc))
    assert rel(z, zc) < 1e-10
    solver = M.ConjGrad(s, precond=B, tolerance=1e-8, maxiter=500)       # device PCG
    B._Aop = s
    solver * r
    t0 = time.time()
    _, cres = ch.pcg(r, 1e-8, 500)
    say('PCG iterations GPU %d, CPU %d (CPU %.1fs, %d threads)'
        % (len(solver.residuals) - 1, len(cres) - 1, time.time() - t0, ch.threads()))
    assert len(solver.residuals) == len(cres)
    assert np.allclose(solver.residuals, cres, rtol=1e-6, atol=0)
    H.close()
    B.close()


def test_emi_3d_nrefs5_reference_default_rings(lib_built):
    """BASELINE config 4's system (emi_3d nrefs=5, N = 278,850) with the EMI
    drivers' own preconditioner call (no parameters: the reference's default
    dict, seed-ring Schwarz on the 8,450 interface seeds' 2-rings): the GPU
    and the host setup give bitwise-equal applies, the cycle without coarse
    scaling is symmetric, and PCG (tolerance 1e-10, src/emi_3d.py:143)
    converges in few iterations."""
    import torch
    M = _M()
    P = M.parameters
    s = M.problems.emi(3, 64, 1e6)
    A = s.scipy()
    Bg = M.precond.get_hazmath_metric_precond_mono(A, s.W, interface_dofs=s.idofs, setup='gpu')
    Bh = M.precond.get_hazmath_metric_precond_mono(A, s.W, interface_dofs=s.idofs, setup='host')
    assert Bg.setup_path == 'gpu' and Bg.level_format(0)['rings']
    r = M.problems.seeded_rhs(s.N)
    assert np.array_equal(Bg * r, Bh * r)
    Bh.close()
    Bs = M.precond.get_hazmath_metric_precond_mono(A, s.W, interface_dofs=s.idofs,
                                                   parameters=dict(P.parameters_metric_default, coarse_scaling=0))
    r1, r2 = torch.as_tensor(r).cuda(), torch.as_tensor(M.problems.seeded_rhs(s.N, 5)).cuda()
    a, c = float(torch.dot(r2, Bs.matvec(r1))), float(torch.dot(r1, Bs.matvec(r2)))
    assert abs(a - c) <= 1e-9 * abs(a)
    Bs.close()
    solver = M.ConjGrad(A, precond=Bg, tolerance=1e-10, maxiter=500)
    solver * r
    say('EMI 3-D nrefs=5, reference default dict (seed rings): PCG iterations %d' % (len(solver.residuals) - 1))
    assert len(solver.residuals) - 1 <= 40
    Bg.close()


def test_emi_3d_nrefs5_block_form(lib_built):
    import torch
    M = _M()
    n = 2 ** (2 + 5 - 1)                                   # src/emi_3d.py:119, nrefs=5
    s = M.problems.emi(3, n, 1e6)
    assert s.N == 278850
    BB = M.precond.get_hazmath_metric_precond(s.blocks, s.W, parameters=M.parameters.parameters_metric_mi355x,
                                              interface_dofs=s.idofs, num_functions=2)
    Bm = BB.monolithic
    A = s.scipy()
    b = [M.problems.seeded_rhs(s.W[0], 1234), M.problems.seeded_rhs(s.W[1], 4321)]
    bb = np.concatenate(b)
    # the same hierarchy on the host (setup = the product's host setup, which
    # tests/test_host_setup.py pins bitwise to the Python oracle)
    seeds = Bm.idofs
    H = M.HostHierarchy(A, idofs=seeds, num_functions=2)
    ch = c_hierarchy(H, A)
    z = (Bm.matvec(torch.as_tensor(bb).cuda())).cpu().numpy()
    assert rel(z, ch.apply(bb)) < 1e-10
    solver = M.ConjGrad(s, precond=BB, tolerance=1e-10, maxiter=500)     # src/emi_3d.py:143
    solver * b
    _, cres = ch.pcg(bb, 1e-10, 500)
    say('EMI 3-D nrefs=5: PCG iterations GPU %d, CPU %d' % (len(solver.residuals) - 1, len(cres) - 1))
    assert len(solver.residuals) == len(cres)
    assert np.allclose(solver.residuals, cres, rtol=1e-6, atol=0)
    assert len(solver.residuals) < 120
    H.close()


def test_emi_3d_nrefs5_reference_default_rings_8_virtual_ranks(lib_built):
    """BASELINE config 4 with the EMI drivers' own call on 8 ranks (VERDICT
    r05 #7): get_hazmath_metric_precond_mono(A, W, interface_dofs) without
    parameters = the default dict's seed rings, row-partitioned over 8 virtual
    ranks (5-hop ghost regions, a halo per ring colour and per rest-GS
    colour).  The gathered apply = the one-GPU apply to 1e-12 and the oracle's
    to 1e-10; the distributed PCG (tolerance 1e-10, src/emi_3d.py:143) takes
    the one-GPU iteration count."""
    import torch
    import mamg_oracle as mo
    M = _M()
    n = M.problems.finest_n(3, 5, 'emi')
    s = M.problems.emi(3, n, 1e6)
    assert s.N == 278850
    A = s.tocsr()
    B = M.precond.get_hazmath_metric_precond_mono(A, s.W, interface_dofs=s.idofs, setup='gpu')
    assert B.level_format(0)['rings']
    r = M.problems.seeded_rhs(s.N)
    z = B * r
    P = 8
    hs = [M.DistMetricAMG(A, s.W, idofs=s.idofs, parameters=M.parameters.parameters_metric_default, rank=p,
                          nranks=P, comm_id=None, rep_nodes=4096) for p in range(P)]
    rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
    zs = [torch.zeros_like(x) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, zs)
    torch.cuda.synchronize()
    zd = np.zeros(s.N)
    for hh, zl in zip(hs, zs):
        zl = zl.cpu().numpy()
        zd[hh.o0:hh.o1] = zl[:hh.nloc]
        zd[s.nv + hh.o0:s.nv + hh.o1] = zl[hh.nloc:]
    h = mo.setup(A, mo.Params(AMG_type='UA', cycle_type='W', smoother='SGS', relaxation=1.2, coarse_scaling=1,
                              aggregation_type='HEM', strong_coupled=0.1, Schwarz_levels=1, Schwarz_mmsize=100,
                              Schwarz_maxlvl=2, Schwarz_type=3, num_functions=2), idofs=s.idofs)
    e1, eo = rel(zd, z), rel(zd, h.apply(r))
    cg1 = M.ConjGrad(A, precond=B, tolerance=1e-10, maxiter=500)
    cg1 * r
    dcg = M.DistConjGrad.for_handles(hs, tolerance=1e-10, maxiter=500)
    dcg.solve([x.clone() for x in rs])
    say('EMI 3-D nrefs=5, default dict (seed rings), 8 virtual ranks: vs one GPU %.2e, vs oracle %.2e, '
        'PCG %d (one GPU %d)' % (e1, eo, len(dcg.residuals) - 1, len(cg1.residuals) - 1))
    assert e1 < 1e-12 and eo < 1e-10
    assert len(dcg.residuals) == len(cg1.residuals)
    for hh in hs:
        hh.close()
    B.close()


def test_emi_3d_nrefs5_node_aligned_8_virtual_ranks(lib_built):
    """BASELINE config 4 (emi_3d nrefs=5 gamma=1e6 row-partitioned over 8
    GPUs): the interface seeds with node-aligned blocks (Schwarz_maxlvl 0),
    GPU setup; one GPU against the C cycle on the same hierarchy, and the
    8-rank row partition (virtual ranks: the RCCL path's counts, offsets and
    kernels, device copies for the exchanges) against the one-GPU apply."""
    import torch
    M = _M()
    n = M.problems.finest_n(3, 5, 'emi')
    s = M.problems.emi(3, n, 1e6)
    assert s.N == 278850
    A = s.tocsr()
    kw = dict(num_functions=2, Schwarz_maxlvl=0)
    B = M.MetricAMG(A, s.W, idofs=s.idofs, setup='gpu', **kw)
    r = M.problems.seeded_rhs(s.N)
    z = B.matvec(torch.as_tensor(r).cuda()).cpu().numpy()
    H = M.HostHierarchy(A, idofs=s.idofs, gpu=True, **kw)
    ch = c_hierarchy(H, A)
    assert rel(z, ch.apply(r)) < 1e-10
    P = 8
    hs = [M.DistMetricAMG(A, s.W, idofs=s.idofs, rank=p, nranks=P, comm_id=None, rep_nodes=4096, **kw)
          for p in range(P)]
    rs = [torch.as_tensor(hh.local_slice(r)).cuda() for hh in hs]
    zs = [torch.zeros_like(x) for x in rs]
    M.DistMetricAMG.virtual_apply(hs, rs, zs)
    torch.cuda.synchronize()
    zd = np.zeros(s.N)
    for hh, zl in zip(hs, zs):
        zl = zl.cpu().numpy()
        zd[hh.o0:hh.o1] = zl[:hh.nloc]
        zd[s.nv + hh.o0:s.nv + hh.o1] = zl[hh.nloc:]
    say('EMI 3-D nrefs=5, 8 virtual ranks vs one GPU: %.2e' % rel(zd, z))
    assert rel(zd, z) < 1e-10
    for hh in hs:
        hh.close()
    H.close()
    B.close()


def _relres_pcg(A, apply, b, tol, maxit):
    """PCG stopped on ||r|| / ||b|| (HAZmath linear_stop_type 1,
    src/input_metric.dat:54) with the preconditioner `apply` (the C cycle)."""
    x = np.zeros_like(b)
    r = b.copy()
    z = apply(r)
    d = z.copy()
    rz = r @ z
    bn = np.linalg.norm(b)
    it = 0
    while np.linalg.norm(r) > tol * bn and it < maxit:
        q = A @ d
        al = rz / (d @ q)
        x += al * d
        r -= al * q
        z = apply(r)
        rz2 = r @ z
        d = z + (rz2 / rz) * d
        rz = rz2
        it += 1
    return x, it


@pytest.mark.parametrize('radius', [0.0, 1.0])
def test_emi_3d1d_gamma_sweep(lib_built, radius):
    """BASELINE config 5 on one GPU: the 3D-1D system (src/emi_3d1d.py:99-167)
    on a 49^3 tissue cube with the synthetic branched neuron, gamma swept
    1e0..1e8 (run_emi_3d1d.sh:5-17), profile parameters_metric_3d1d (additive
    overlapping Schwarz on the 1-D seeds' 2-rings).  Per gamma, against the
    oracle: the host setup's hierarchy (bitwise the Python oracle's,
    tests/test_host_setup.py) run by the oracle's C cycle (oracle/vcycle_ref.c)
    equals one GPU apply to 1e-10 (1e-8 at gamma >= 1e8); the
    PCG with the GPU preconditioner and the PCG with the C cycle (both stopped
    on ||r|| / ||b|| < 1e-6) take the same iterations and reach solutions
    equal to 1e-6; the counts stay gamma-robust."""
    M = _M()
    P = M.parameters
    its = {}
    for g in (1.0, 1e2, 1e4, 1e6, 1e8):
        s = M.problems.emi_3d1d(48, g, radius)
        A = s.scipy()
        b = M.problems.seeded_rhs(s.N)
        B = M.MetricAMG(A, s.W, idofs=s.idofs, parameters=P.parameters_metric_3d1d)
        H = M.HostHierarchy(A, idofs=s.idofs, parameters=P.parameters_metric_3d1d)
        assert H.num_levels == B.num_levels
        ch = c_hierarchy(H, A)
        tol = 1e-10 if g < 1e8 else 1e-8
        for seed in (1234, 7):
            r = M.problems.seeded_rhs(s.N, seed)
            assert rel(B * r, ch.apply(r)) < tol
        dev = M.ConjGrad(A, precond=B, tolerance=1e-6, maxiter=1000, stop_type=1)
        x = dev * b
        x = x.cpu().numpy() if hasattr(x, 'cpu') else np.asarray(x)
        xo, n_or = _relres_pcg(A, ch.apply, b, 1e-6, 1000)
        n_dev = len(dev.residuals) - 1
        say('emi_3d1d n=48 radius', radius, 'gamma', g, 'N', s.N, 'PCG its GPU', n_dev, 'C oracle', n_or)
        assert n_dev == n_or
        assert np.linalg.norm(b - A @ x) <= 1e-6 * np.linalg.norm(b)
        assert rel(x, xo) <= 1e-6
        its[g] = n_dev
        B.close()
        H.close()
    assert max(its.values()) < 200
    assert max(its.values()) <= 3 * min(its.values()), its


def _sweep_worker(rank, world, port, q):
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
        import metric_amg_examples_amd.drivers as D

        def gather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out
        torch.cuda.set_device(0)
        units = D.sweep_units([0.0, 1.0], [1.0, 1e4, 1e8])
        rows, _, _ = D.run_sweep(units, lambda u: D.solve_3d1d_unit(16, u[0], u[1], device=0), rank, world, gather)
        q.put((rank, rows))
    finally:
        dist.destroy_process_group()


def test_emi_3d1d_sweep_two_processes(lib_built):
    """BASELINE config 5 on N ranks (drivers.emi_3d1d_sweep): the radius x
    gamma solves of run_emi_3d1d.sh:5-17 sharded over two processes on the
    GPU (units k % 2), rows gathered over gloo.  Every unit's PCG iteration
    count equals the oracle's (the host setup's hierarchy run by the C cycle,
    PCG stopped on ||r|| / ||b|| < 1e-6) and its true relative residual is
    below the tolerance."""
    import socket
    import torch.multiprocessing as mp
    M = _M()
    import metric_amg_examples_amd.drivers as D
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    procs = [ctx.Process(target=_sweep_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    units = D.sweep_units([0.0, 1.0], [1.0, 1e4, 1e8])
    rows = res[0]
    assert [(r['radius'], r['gamma']) for r in rows] == units
    assert [r['rank'] for r in rows] == [k % 2 for k in range(len(units))]
    P = M.parameters
    for (radius, g), row in zip(units, rows):
        s = M.problems.emi_3d1d(16, g, radius)
        A = s.scipy()
        b = M.problems.seeded_rhs(s.N)
        H = M.HostHierarchy(A, idofs=s.idofs, parameters=P.parameters_metric_3d1d)
        ch = c_hierarchy(H, A)
        _, n_or = _relres_pcg(A, ch.apply, b, 1e-6, 1000)
        H.close()
        say('sweep radius', radius, 'gamma', g, 'rank', row['rank'], 'its', row['niters'], 'oracle', n_or)
        assert row['niters'] == n_or
        assert row['relres'] <= 1e-6


def test_bidomain_2d_config1_reference_cli(lib_built, tmp_path):
    """BASELINE config 1 through the reference's own command line
    (`bidomain_2d.py -nrefs 3 -gamma 1 -precond metric_mono`):
    the driver's mesh loop n = 32, 64, 128 (src/bidomain_2d.py:168) with the
    preset the reference's driver passes (parameters_metric_schwarz, src/
    bidomain_3d.py:144-147: UA + HEM + W + SGS + scaling + the level-0 node
    patches) and the manufactured right-hand side.  On every mesh the GPU PCG
    iteration count equals the oracle's restatement of that algorithm on the
    same right-hand side, and the iters file has the reference's schema."""
    import importlib
    M = _M()
    D = importlib.import_module('metric_amg_examples_amd.drivers')
    P = M.parameters
    rows = D.bidomain(['-nrefs', '3', '-gamma', '1', '-precond', 'metric_mono', '-results', str(tmp_path)], 2)
    assert [r[0] for r in rows] == [2 * 33 ** 2, 2 * 65 ** 2, 2 * 129 ** 2]
    d = P.parameters_metric_schwarz
    op = mo.Params(AMG_type='UA', cycle_type='W', aggregation_type='HEM', smoother='SGS',
                   max_levels=d['max_levels'], maxit=d['maxit'], relaxation=d['relaxation'],
                   presmooth_iter=d['presmooth_iter'], postsmooth_iter=d['postsmooth_iter'],
                   coarse_dof=d['coarse_dof'], strong_coupled=d['strong_coupled'],
                   coarse_scaling=d['coarse_scaling'], Schwarz_levels=d['Schwarz_levels'],
                   Schwarz_mmsize=d['Schwarz_mmsize'], Schwarz_maxlvl=d['Schwarz_maxlvl'],
                   Schwarz_type=d['Schwarz_type'], num_functions=2)
    for (N, niters, cond, dt, r, h), n in zip(rows, (32, 64, 128)):
        s = M.problems.bidomain(2, n, 1.0)
        b = M.problems.bidomain_mms_rhs(2, n, 1.0, 2.0, 3.0)
        t0 = time.time()
        hh = mo.setup(s.scipy(), op, idofs=s.idofs)
        ref = mo.pcg(s.scipy(), hh, b, 1e-8, 500)
        say('config 1 n=%d: GPU %d iterations, oracle %d (%.1fs), timeKSP %.3fs' % (n, niters, ref.niters,
                                                                                time.time() - t0, dt))
        assert niters == ref.niters, (n, niters, ref.niters)
        assert abs(r - ref.residuals[-1]) <= 1e-6 * ref.residuals[-1]
    files = sorted((tmp_path / 'bidomain_2d').glob('iters_precondmetric_mono_*.txt'))
    assert len(files) == 1, files
    lines = files[0].read_text().split('\n')
    assert lines[0] == 'ndofs niters cond timeKSP r h' and len([x for x in lines[1:] if x]) == 3
