#!/usr/bin/env python3
"""Benchmark: metric-AMG preconditioner applications (one V-cycle each) per
second and achieved HBM GB/s on the bidomain_3d nrefs=6 system
(BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--nrefs 6] [--dim 3]
    torchrun --nproc-per-node N bench.py --gpus N ...   (multi-GPU)

A step = one preconditioner application z = B r (one V-cycle from x0 = 0) on
a resident seeded r (uniform(-1,1), seed 1234) -- the unit of work of the
reference's hot loop (`BB * r` inside ConjGrad, src/bidomain_3d.py:149-150).
The timed region runs K applies kernel by kernel on one stream with HIP
events around the two dominant kernels of every step (level-0 residual SpMV
and the fused prolongation + post-smoothing kernel), bracketed by barrier +
synchronize; `roofline` is the one with the larger time.  value = K / max-over-ranks wall time
(applies of the whole problem per second).
N = 1: the whole hierarchy on one GPU (BSR2 layout, hipGraph replay also
reported).  N > 1: the same problem row-partitioned over N GPUs (one process
per GPU, RCCL halo exchange over xGMI; strong scaling).
The cpu_baseline leg (rank 0, N = 1) times the oracle's C restatement
(oracle/vcycle_ref.c) of the same cycle on the same hierarchy on the host.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "V-cycle applies/sec + HBM GB/s, bidomain_3d nrefs=6 @1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md); 6290 measured copy
CLASS_NAMES = ['L0_resid', 'L0_smooth_spmv', 'L0_smoother', 'L0_restrict', 'L0_prolong',
               'coarse_levels', 'coarsest_dense', 'misc', 'comm']


PROFILE_NAMES = {'jacobi': 'mi355x_sa_v: nodal SA V-cycle, node-block Jacobi',
                 'poly': 'mi355x_poly: nodal SA V-cycle, Chebyshev steps of node-block Jacobi',
                 'sgs': 'mi355x_sgs: nodal SA V-cycle, multicolour node-block SGS',
                 'gs': 'nodal SA V-cycle, multicolour node-block GS'}


def log(*a):
    print('[bench]', *a, file=sys.stderr, flush=True)


def breakdown_dict(kms, cbytes, ms_all):
    out = {nm: {'ms': round(kms[i], 4), 'GB': round(cbytes[i] / 1e9, 4),
                'GBps': round(cbytes[i] / 1e9 / (kms[i] * 1e-3), 1) if kms[i] > 0 else None}
           for i, nm in enumerate(CLASS_NAMES)}
    out['instrumented_ms_per_apply'] = round(ms_all, 4)
    return out


def device_src_sha():
    import hashlib
    with open(os.path.join(ROOT, 'metric-amg-examples_amd', 'csrc', 'device.hip'), 'rb') as f:
        return hashlib.sha256(f.read()).hexdigest()


def rss_gb():
    """peak resident set size of this process (GB)."""
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6


def cpu_quota():
    """CPUs the cgroup lets this process use (cpu.max / cfs quota), or None."""
    try:
        q, p = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            return int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
        p = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
        if q > 0:
            return q / p
    except (OSError, ValueError):
        pass
    return None


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return None


def one_gpu_check(args, M, B, r, z, r_full, sysm, prof, dev, rdev, gloo, rank, world, dist_res, barrier, allsum):
    """N > 1: z (this rank's slice of the distributed B r) and the distributed
    PCG residual history against rank 0's one-GPU preconditioner on the same
    matrix; returns the record (every rank computes the same one)."""
    import torch
    import torch.distributed as tdist
    M.release_setup_cache()                 # the distributed setup's cached blocks
    barrier()
    t0 = time.time()
    n = M.problems.finest_n(args.dim, args.nrefs, args.problem)
    N = sysm.N
    z1 = torch.empty(N, dtype=torch.float64, device=rdev)
    meta = [None]
    if rank == 0:
        A0 = M.problems.bidomain_device(args.dim, n, args.gamma, device=dev)
        B1 = M.MetricAMG(A0, sysm.W, idofs=sysm.idofs, num_functions=2, device=dev.index, setup='gpu', **prof)
        rf = torch.as_tensor(r_full).to(dev)
        zz = torch.zeros_like(rf)
        B1.apply_device(rf, zz)
        res1 = None
        if dist_res is not None:
            B1._Aop = sysm
            cg = M.ConjGrad(sysm, precond=B1, tolerance=1e-8, maxiter=500)
            cg.solve_device(rf)
            res1 = [float(v) for v in cg.residuals]
        torch.cuda.synchronize(dev)
        z1.copy_(zz)
        meta = [{'residuals': res1, 'setup_s': round(time.time() - t0, 3)}]
        B1.close()
        del A0, rf, zz
        M.release_setup_cache()
    tdist.broadcast(z1, src=0)
    tdist.broadcast_object_list(meta, src=0)
    z1 = z1.to(dev)
    nv = B.nv
    zl = torch.cat([z1[B.o0:B.o1], z1[nv + B.o0:nv + B.o1]])
    num = allsum(float(((z - zl) ** 2).sum()))
    den = allsum(float((zl ** 2).sum()))
    rz_d = allsum(float((r * z).sum()))
    rz_1 = allsum(float((r * zl).sum()))
    del z1, zl
    out = {'z_rel_vs_1gpu': float(np.sqrt(num / den)) if den > 0 else None,
           'rz_dist': rz_d, 'rz_1gpu': rz_1, 'seed': 1234,
           'one_gpu_setup_s': meta[0]['setup_s'],
           'note': 'rank 0 set up the one-GPU preconditioner on the same matrix (A_0 regenerated in its HBM) '
                   'after the timed region; z = B r of the %d ranks gathered against its z' % world}
    res1 = meta[0]['residuals']
    if res1 is not None and dist_res is not None:
        out['pcg_niters_1gpu'] = len(res1) - 1
        out['pcg_niters_dist'] = len(dist_res) - 1
        out['pcg_niters_equal'] = len(res1) == len(dist_res)
        out['max_rel_residual_diff'] = float(max(abs(a - b) / b for a, b in zip(dist_res, res1))) \
            if len(res1) == len(dist_res) else None
    barrier()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--dim', type=int, default=3)
    ap.add_argument('--nrefs', type=int, default=6)
    ap.add_argument('--gamma', type=float, default=1e6)
    ap.add_argument('--problem', choices=('bidomain', 'emi'), default='bidomain',
                    help='bidomain (BASELINE configs 1-3) or emi (config 4: emi_3d nrefs=5, interface seeds '
                         'with node-aligned blocks, Schwarz_maxlvl 0)')
    ap.add_argument('--rep-nodes', type=int, default=32768,
                    help='multi-GPU: replicate levels with <= this many nodes')
    ap.add_argument('--cpu-sample', type=int, default=10,
                    help='CPU baseline: timed applies after 2 warm-ups, median reported (0: skip)')
    ap.add_argument('--no-breakdown', action='store_true')
    ap.add_argument('--pcg', type=int, default=1,
                    help='run one full PCG solve (N = 1: device PCG; N > 1: DistConjGrad over RCCL, its '
                         'iterations and residual history checked against the one-GPU solve)')
    ap.add_argument('--check-1gpu', type=int, default=1,
                    help='N > 1: rank 0 also sets up the one-GPU preconditioner on the same matrix after the '
                         'timed region; the line carries z = B r gathered over the ranks against its z, and the '
                         'distributed PCG against its PCG (north star: equal iteration count at 1/2/4/8)')
    ap.add_argument('--cpu-pcg', type=int, default=1,
                    help='N = 1: also run the CPU PCG (oracle C cycle + SpMV, host cores) on the same '
                         'hierarchy and report its iteration count next to the GPU one')
    ap.add_argument('--compare-profiles', type=int, default=1,
                    help='N = 1: also set up and solve with the multicolour-SGS profile (iterations, seconds)')
    ap.add_argument('--setup', choices=('gpu', 'host'), default='gpu',
                    help='N = 1 hierarchy construction: GPU setup (default) or host setup + upload')
    ap.add_argument('--smoother', choices=('jacobi', 'poly', 'sgs', 'gs'), default='jacobi',
                    help='level smoother: node-block Jacobi (mi355x_sa_v), Chebyshev steps of it (poly), '
                         'or multicolour node-block SGS / GS')
    ap.add_argument('--poly-degree', type=int, default=2)
    ap.add_argument('--scaling', type=int, default=0, help='coarse-grid correction scaling (coarse_scaling ON)')
    ap.add_argument('--cycle', choices=('V', 'W'), default='V')
    ap.add_argument('--dist-graph', type=int, default=1,
                    help='N > 1 over RCCL: time hipGraph replays of the apply (checked bitwise against eager first)')
    ap.add_argument('--exchange', choices=('rccl', 'gloo'), default='rccl',
                    help='N > 1 transport: RCCL (default), or the host-staged gloo exchange '
                         '(mamg_dist_set_exchange; runs several ranks on one GPU, for rehearsals)')
    ap.add_argument('--host-matrix', action='store_true',
                    help='N > 1: generate the global A_0 on the host of every rank (before round 4) instead of '
                         'in each rank\'s HBM')
    ap.add_argument('--compare-host-setup', action='store_true',
                    help='also time the host setup of the same hierarchy (N = 1)')
    args = ap.parse_args()
    prof = dict(smoother={'jacobi': 3, 'poly': 12, 'sgs': 11, 'gs': 10}[args.smoother], coarse_scaling=args.scaling,
                cycle_type={'V': 1, 'W': 2}[args.cycle], poly_degree=args.poly_degree,
                Schwarz_type={'sgs': 7, 'gs': 7}.get(args.smoother, 4))

    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.exchange == 'gloo' and torch.cuda.device_count() > 0:
        local %= torch.cuda.device_count()      # rehearsal: several ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    gloo = world > 1 and args.exchange == 'gloo'
    if world > 1:
        import torch.distributed as dist
        if gloo:
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=dev)
    rdev = torch.device('cpu') if gloo else dev        # device of the timing reductions

    import metric_amg_examples_amd as M

    n = M.problems.finest_n(args.dim, args.nrefs, args.problem)
    t0 = time.time()
    A0dev = None
    if args.problem == 'emi':      # src/emi_3d.py:119-144 (split cube, trace coupling, interface seeds)
        sysm = M.problems.emi(args.dim, n, args.gamma)
        prof['Schwarz_maxlvl'] = 0
    elif world > 1 and not args.host_matrix:
        # N > 1: every rank generates A_0 in its own HBM (mamg_gen_bidomain_device,
        # bitwise the host generator's); no rank holds the global matrix on the
        # host (13-14 GB of RSS per rank before round 4)
        A0dev = M.problems.bidomain_device(args.dim, n, args.gamma, device=dev)
        sysm = M.problems.bidomain_meta(args.dim, n, int(A0dev[1].numel()))
    else:
        sysm = M.problems.bidomain(args.dim, n, args.gamma)
    Aop = sysm.tocsr() if args.problem == 'emi' else sysm   # the operator PCG and the setup share
    t_gen = time.time() - t0
    log('rank %d: generated %dD n=%d N=%d nnz=%d in %.1fs%s' % (rank, args.dim, n, sysm.N, sysm.nnz, t_gen,
                                                               ' (in HBM)' if A0dev is not None else ''))
    stream = torch.cuda.current_stream(dev)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
            torch.cuda.synchronize(dev)

    def allmax(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=rdev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return t.item()

    def allsum(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=rdev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM)
        return t.item()

    r_full = M.problems.seeded_rhs(sysm.N)
    H = None
    setup_info = {}
    if world == 1:
        if args.setup == 'host':
            t0 = time.time()
            H = M.HostHierarchy(sysm, idofs=sysm.idofs, num_functions=2, device=local, **prof)
            t_setup = time.time() - t0
            t0 = time.time()
            B = M.MetricAMG.from_host(H, sysm.W)
            t_upload = time.time() - t0
            setup_info = {'path': 'host', 'host_setup_s': round(t_setup, 3), 'upload_s': round(t_upload, 3)}
        else:
            # GPU setup: A0 copied to HBM once, hierarchy and apply layouts
            # built by gfx950 kernels (bitwise equal to the host setup)
            torch.cuda.synchronize(dev)
            t0 = time.time()
            B = M.MetricAMG(Aop, sysm.W, idofs=sysm.idofs, num_functions=2, device=local, setup='gpu', **prof)
            t_setup = time.time() - t0
            setup_info = {'path': 'gpu', 'wall_s': round(t_setup, 3), 'phases_ms': B.setup_timings}
            if args.compare_host_setup:
                t0 = time.time()
                Hc = M.HostHierarchy(sysm, idofs=sysm.idofs, num_functions=2, device=local, **prof)
                setup_info['host_setup_s'] = round(time.time() - t0, 3)
                Hc.close()
        levels = None
        layout = B.layout
        r = torch.as_tensor(r_full).to(dev)
    else:
        uid = [M.DistMetricAMG.unique_id() if (rank == 0 and not gloo) else None]
        torch.distributed.broadcast_object_list(uid, src=0)
        t0 = time.time()
        B = M.DistMetricAMG(A0dev if A0dev is not None else sysm, sysm.W, idofs=sysm.idofs, rank=rank,
                            nranks=world, comm_id=uid[0], rep_nodes=args.rep_nodes, num_functions=2, device=local,
                            exchange='gloo' if gloo else None, **prof)
        t_setup = time.time() - t0
        A0dev = None                       # the rank keeps only its operators
        torch.cuda.empty_cache()
        setup_info = {'path': 'deterministic setup replicated on every rank (GPU setup; host setup if the '
                              'profile is unsupported) + rank-local upload',
                      'A0': 'host' if hasattr(sysm, 'indptr') else 'generated in HBM per rank',
                      'wall_s': round(t_setup, 3), 'host_rss_gb_max_rank': round(allmax(rss_gb()), 2),
                      # eager distributed apply: what rank 0 issues per apply
                      'apply_launches_rank0': B.apply_launches}
        levels = None
        layout = 'bsr2-dist'
        r = torch.as_tensor(B.local_slice(r_full)).to(dev)
        log('rank %d: nodes [%d, %d) of %d, setup+upload %.1fs' % (rank, B.o0, B.o1, B.nv, t_setup))
    z = torch.zeros_like(r)

    # warmup
    for _ in range(max(1, args.warmup)):
        B.apply_device(r, z, stream)
    B.time_apply(r, z, max(1, args.warmup), 0, stream)
    barrier()

    # ---- N > 1 over RCCL: the apply replayed from a hipGraph (RCCL calls
    # inside the capture) when every rank's graph apply is bitwise its eager
    # apply; otherwise the eager path (the line records which and why)
    use_graph = False
    graph_info = None
    if world > 1 and not gloo and args.dist_graph:
        # capture on every rank first (nothing launched), agree, then launch:
        # a graph's RCCL calls wait for every peer's
        zg = torch.full_like(z, float('nan'))
        gerr = B.prepare_graph(r, zg) or B.prepare_graph(r, z)
        captured = allsum(0.0 if gerr is None else 1.0) == 0.0
        same = False
        if captured:
            B.apply_device(r, z, stream)
            B.apply_graph(r, zg, stream)
            torch.cuda.synchronize(dev)
            same = allsum(0.0 if bool(torch.equal(z, zg)) else 1.0) == 0.0
        use_graph = captured and same
        graph_info = {'used': use_graph, 'captured_all_ranks': captured, 'bitwise_equal_eager_all_ranks': same,
                      'rank0_error': gerr}
        del zg
        if use_graph:
            B.time_apply(r, z, max(1, args.warmup), 2, stream)
        barrier()

    # ---- timed region: K applies (eager with events around the dominant
    # kernels; N > 1: graph replays when checked above)
    t0 = time.perf_counter()
    ms_ev, kms, cbytes = B.time_apply(r, z, args.steps, 2 if use_graph else 0, stream)
    barrier()
    wall = allmax(time.perf_counter() - t0)
    ms_per_step = 1e3 * wall / args.steps
    value = args.steps / wall
    apply_bytes = allsum(B.apply_bytes)
    if use_graph:
        # the eager path on the same handles, for the record, and its kernel
        # events (graph replays carry none) for the roofline
        barrier()
        t0 = time.perf_counter()
        _, kms, cbytes = B.time_apply(r, z, args.steps, 0, stream)
        barrier()
        wall_e = allmax(time.perf_counter() - t0)
        graph_info.update(ms_per_step_graph=round(ms_per_step, 4),
                          ms_per_step_eager=round(1e3 * wall_e / args.steps, 4))
    elif graph_info is not None:
        graph_info.update(ms_per_step_graph=None, ms_per_step_eager=round(ms_per_step, 4))

    graph_ms = None
    if world == 1:                          # hipGraph replay of the same work
        barrier()
        g0 = torch.cuda.Event(enable_timing=True)
        g1 = torch.cuda.Event(enable_timing=True)
        g0.record(stream)
        for _ in range(args.steps):
            B.apply_device(r, z, stream)
        g1.record(stream)
        barrier()
        graph_ms = round(g0.elapsed_time(g1) / args.steps, 4)

    breakdown = None
    if not args.no_breakdown:
        ms_all, kms_all, _ = B.time_apply(r, z, max(3, args.steps // 4), 1, stream)
        barrier()
        breakdown = breakdown_dict(kms_all, cbytes, ms_all)

    pcg = None
    gpu_res = None
    if args.pcg and world == 1:
        B._Aop = Aop
        solver = M.ConjGrad(Aop, precond=B, tolerance=1e-8, maxiter=500)
        torch.cuda.synchronize(dev)
        t0 = time.time()
        solver * r                      # right-hand side resident in HBM (as the timed applies)
        torch.cuda.synchronize(dev)
        tp = time.time() - t0
        gpu_res = list(solver.residuals)
        pcg = {'niters': len(solver.residuals) - 1, 'residual': solver.residuals[-1],
               'seconds': round(tp, 4), 'setup_s': round(t_setup, 4),
               'setup_plus_pcg_s': round(tp + t_setup, 4),
               'note': 'cbc.block ConjGrad, tolerance 1e-8 absolute on sqrt(<r,Br>), maxiter 500 '
                       '(src/bidomain_3d.py:149), device-resident (b, x in HBM; one hipGraph per '
                       'iteration, scalars on the device); timeKSP-style: setup + solve'}
    elif args.pcg:
        solver = M.DistConjGrad.for_handles(B, stream=stream, tolerance=1e-8, maxiter=500)
        barrier()
        t0 = time.perf_counter()
        solver.solve([r.clone()])
        barrier()
        pcg = {'niters': len(solver.residuals) - 1, 'residual': solver.residuals[-1],
               'seconds': round(allmax(time.perf_counter() - t0), 3),
               'note': 'DistConjGrad: cbc.block ConjGrad on the row-partitioned slices, dots all-reduced '
                       '(src/bidomain_3d.py:149)'}
        gpu_res = list(solver.residuals)

    # ---- N > 1 parity against one GPU: rank 0 builds the
    # single-GPU preconditioner on the same matrix (A_0 regenerated in its HBM)
    # after everything timed; z = B r and the PCG solve are compared with the
    # distributed ones
    check_1gpu = None
    if world > 1 and args.check_1gpu and args.problem == 'bidomain':
        check_1gpu = one_gpu_check(args, M, B, r, z, r_full, sysm, prof, dev, rdev, gloo, rank, world,
                                   gpu_res if args.pcg else None, barrier, allsum)

    # ---- the reference's smoother family on the GPU (multicolour SGS +
    # coarse-grid scaling): iterations and time to solution next to the default
    profiles = None
    if args.compare_profiles and world == 1 and args.pcg:
        profiles = []
        for name, kw in (('mi355x_poly (Chebyshev degree 2 of node-block Jacobi)', dict(smoother=12)),
                         ('mi355x_sa_v (node-block Jacobi)', dict(smoother=3)),
                         ('mi355x_sgs (multicolour node-block SGS, coarse scaling ON)',
                          dict(smoother=11, coarse_scaling=1, Schwarz_type=7)),
                         ('reference family: UA + parallel HEM + W-cycle + multicolour SGS + coarse scaling, '
                          'strong_coupled 0.1 (src/amg_parameters.py:67-89)',
                          dict(AMG_type=1, aggregation_type=5, cycle_type=2, smoother=11, coarse_scaling=1,
                               strong_coupled=0.1, Schwarz_type=7)),
                         ('parameters_standard: UA + sequential Vanek-Mandel-Brezina (VMB) + W-cycle + '
                          'multicolour SGS + coarse scaling (src/amg_parameters.py:16-36)',
                          dict(AMG_type=1, aggregation_type=1, cycle_type=2, smoother=11, coarse_scaling=1,
                               strong_coupled=0.1, Schwarz_type=7)),
                         ('reference family, coarse_dof 2048 (dense solve instead of the launch-bound W bottom)',
                          dict(AMG_type=1, aggregation_type=5, cycle_type=2, smoother=11, coarse_scaling=1,
                               strong_coupled=0.1, Schwarz_type=7, coarse_dof=2048)),
                         ('mi355x_patch: the reference\'s level-0 smoother (symmetric multiplicative Schwarz on '
                          'the overlapping 1-ring node patches, SCHWARZ_PATCHES), node-block Jacobi below',
                          dict(smoother=3, Schwarz_type=6)),
                         ('reference family with its level-0 node-patch Schwarz: UA + parallel HEM + W-cycle + '
                          'SGS + coarse scaling + SCHWARZ_PATCHES, coarse_dof 2048',
                          dict(AMG_type=1, aggregation_type=5, cycle_type=2, smoother=11, coarse_scaling=1,
                               strong_coupled=0.1, Schwarz_type=6, coarse_dof=2048)),
                         ('parameters_metric_schwarz verbatim (the reference preset: UA + HEM + W + SGS + scaling + '
                          'SCHWARZ_SYMMETRIC 1-rings = SCHWARZ_PATCHES, strong_coupled 0.1, coarse_dof 100)',
                          dict(AMG_type=1, aggregation_type=5, cycle_type=2, smoother=11, coarse_scaling=1,
                               strong_coupled=0.1, Schwarz_type=6, relaxation=1.2)),):
            if (kw['smoother'] == prof['smoother'] and kw.get('coarse_scaling', 0) == prof['coarse_scaling']
                    and kw.get('aggregation_type', 2) == 2 and kw.get('Schwarz_type', 4) == prof['Schwarz_type']):
                continue
            torch.cuda.synchronize(dev)
            t0 = time.time()
            kw = dict(kw, Schwarz_maxlvl=prof.get('Schwarz_maxlvl', 1))
            try:
                B2 = M.MetricAMG(Aop, sysm.W, idofs=sysm.idofs, num_functions=2, device=local, setup='gpu', **kw)
            except M._lib.MamgError as e:      # e.g. a GPU SpGEMM row beyond its widest table
                profiles.append({'profile': name, 'error': str(e)})
                continue
            torch.cuda.synchronize(dev)
            ts = time.time() - t0
            z2 = torch.zeros_like(r)              # z keeps the default profile's apply (CPU check)
            ms2, _, _ = B2.time_apply(r, z2, 5, 0, stream)
            s2 = M.ConjGrad(Aop, precond=B2, tolerance=1e-8, maxiter=500)
            B2._Aop = Aop
            torch.cuda.synchronize(dev)
            t0 = time.time()
            s2 * r
            torch.cuda.synchronize(dev)
            tp2 = time.time() - t0
            profiles.append({'profile': name, 'niters': len(s2.residuals) - 1, 'pcg_s': round(tp2, 4),
                             'setup_s': round(ts, 4), 'setup_plus_pcg_s': round(ts + tp2, 4),
                             'ms_per_apply': round(ms2, 4),
                             'setup_phases_ms': {k: round(v, 1) for k, v in B2.setup_timings.items()}})
            B2.close()
            del s2, z2
            # a closed handle's VRAM (~20 GB; ~80 GB with node patches) is reclaimed by the
            # driver asynchronously, and the next setup in the process can stall 3-6 s until
            # that is done (bench/prof_patch_setup.py --sequence), so the next
            # profile starts after a pause, outside every timed region
            torch.cuda.synchronize(dev)
            time.sleep(5.0)

    # ---- CPU baseline: oracle C restatement on the same hierarchy, host cores
    cpu = None
    c_cycle = args.smoother in ('jacobi', 'poly') and not args.scaling   # what vcycle_ref.c restates
    if rank == 0 and world == 1 and args.cpu_sample > 0 and c_cycle:
        sys.path.insert(0, os.path.join(ROOT, 'oracle'))
        import cref
        import mamg_oracle as mo
        if H is None:       # same hierarchy bits, from the GPU setup copied back
            H = M.HostHierarchy(sysm, idofs=sysm.idofs, num_functions=2, device=local, gpu=True, **prof)
        lv = [H.level(l, with_A=(l > 0)) for l in range(H.num_levels)]
        A0 = Aop.tocsr() if args.problem == 'emi' else sysm
        lv[0]['A'] = (A0.indptr, A0.indices, A0.data, (sysm.N, sysm.N))
        poly = None
        if args.smoother == 'poly':
            poly = mo.poly_weights(mo.Params(smoother='POLY', poly_degree=args.poly_degree,
                                             relaxation=B.params.relaxation, poly_ratio=B.params.poly_ratio))
        ch = cref.CHierarchy(lv, wcycle=args.cycle == 'W', poly=poly)
        # every CPU this process may use: the affinity set, capped by the
        # cgroup quota when one is set (all the host's cores)
        aff = len(os.sched_getaffinity(0))
        quota = cpu_quota()
        nthr = max(1, min(aff, int(quota))) if quota else aff
        ch.set_threads(nthr)
        for _ in range(2):
            ch.apply(r_full)                                 # warm-ups (page-in, thread pool)
        times = []
        for _ in range(args.cpu_sample):
            t0 = time.time()
            zc = ch.apply(r_full)
            times.append(time.time() - t0)
        tc = float(np.median(times))
        zg = z.cpu().numpy()
        err = float(np.linalg.norm(zc - zg) / np.linalg.norm(zc))
        cpu = {'value': round(1.0 / tc, 4), 'unit': 'V-cycle applies/s', 'cores': ch.threads(),
               'kind': 'port', 'nproc': os.cpu_count(), 'affinity': aff, 'cgroup_cpu_quota': quota,
               'cpu_model': cpu_model(), 'apply_s': [round(t, 4) for t in times],
               'sample': 'median of %d applies after 2 warm-ups of the full nrefs=%d hierarchy '
                         '(oracle/vcycle_ref.c, OpenMP, %d threads), GPU-vs-CPU rel diff %.1e'
                         % (args.cpu_sample, args.nrefs, ch.threads(), err)}
        if args.cpu_pcg and pcg is not None:
            # N1: PCG iteration count of the CPU path (same hierarchy bits,
            # C cycle + C SpMV) against the GPU's (src/bidomain_3d.py:149-157)
            t0 = time.time()
            _, cres = ch.pcg(r_full, 1e-8, 500)
            pcg['cpu_pcg'] = {'niters': len(cres) - 1, 'seconds': round(time.time() - t0, 2),
                              'max_rel_residual_diff': float(max(abs(a - b) / b for a, b in
                                                                 zip(gpu_res, cres))) if len(cres) == len(gpu_res)
                              else None,
                              'threads': ch.threads()}
        del ch, lv
    if H is not None and levels is None:
        levels = [[s['n'], s['nnzA']] for s in (H.sizes(l) for l in range(H.num_levels))]

    # measured HBM bytes per launch of the two dominant kernels (rocprofv3
    # FETCH_SIZE + WRITE_SIZE passes, calibrated; profiles/traffic.json,
    # written by scripts/traffic.py from the PMC CSVs of this config).  Used
    # only when it was measured on this kernel source (device.hip sha256)
    # and this layout; the line carries its provenance either way.
    fmt0 = B.level_format(0) if world == 1 and layout == 'bsr2' else {}
    kregion = B.kregion if world == 1 and layout == 'bsr2' else None
    post_mode = 'k' if (fmt0.get('post_k') or world > 1) else 'merged'   # rank-local K by default
    a0_mode = 'half' if fmt0.get('half') else 'sell'
    traffic, traffic_src = {}, None
    tpath = os.path.join(ROOT, 'profiles', 'traffic.json')
    src_sha = device_src_sha()
    if os.path.exists(tpath) and world == 1:
        try:
            tj = json.load(open(tpath))
            ok = (tj.get('N') == sysm.N and tj.get('layout') == layout and tj.get('post', 'merged') == post_mode
                  and tj.get('a0', 'sell') == a0_mode)
            if ok and tj.get('device_src_sha256') == src_sha:
                traffic = tj.get('kernels', {})
                traffic_src = 'profiles/traffic.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of ' \
                              'this kernel source, device.hip sha256 %s)' % src_sha[:16]
            else:
                traffic_src = 'not used: profiles/traffic.json was measured on another kernel source or config ' \
                              '(device.hip sha256 %s vs %s)' % (str(tj.get('device_src_sha256'))[:16], src_sha[:16])
        except (OSError, ValueError):
            traffic = {}

    rk = 'hsell2_kernel' if (fmt0.get('half') or world > 1) else ('sell2_kernel' if fmt0.get('sell') else 'bsr2_kernel')
    if layout == 'csr':
        names = ('csr_kernel<*,RESID,0>', 'csr_kernel<*,BJAC/JACOBI,0>')
    elif post_mode == 'k':
        names = ('%s<RESID,...,0>' % rk,
                 'msell_kernel<2,5,KPOST,...,0>' if (fmt0.get('post_sell') or world > 1) else 'bsr2_kernel<KPOST,...,0>')
    else:
        names = ('%s<RESID,...,0>' % rk,
                 'bsr2_post_kernel<8,...,0>' if fmt0.get('post_fused', True) else 'bsr2_kernel<*,BJAC,...,0>')
    descr = ('level-0 residual r = b - A0 x', 'level-0 prolongation + post-smoothing '
             + ('z = x1 + W r1 + K e, K = P - W (A P)' if post_mode == 'k'
                else 'z = x1 + P e + W (r1 - (AP) e)'))
    if args.smoother in ('sgs', 'gs'):     # the smoothing class is the colour sweeps
        names = (names[0], 'gs2_kernel<VL,SYM>, one launch per colour')
        descr = (descr[0], 'level-0 multicolour node-block %s sweeps (pre + post)' % args.smoother.upper())
    rooflines = []
    for c, key in ((0, 'L0_resid'), (1, 'L0_smooth_spmv')):
        if kms[c] <= 0:
            continue
        ach = cbytes[c] / 1e9 / (kms[c] * 1e-3)
        rooflines.append({
            'bound': 'hbm', 'kernel': '%s (%s)%s' % (descr[c], names[c], '' if world == 1 else ', rank 0 slice'),
            'achieved': round(ach, 1), 'peak': HBM_PEAK_GBPS, 'unit': 'GB/s',
            'frac': round(ach / HBM_PEAK_GBPS, 4), 'traffic': traffic.get(key), 'traffic_source': traffic_src,
            'bytes_per_launch': cbytes[c], 'ms_per_launch': round(kms[c], 4)})
    roofline = max(rooflines, key=lambda r: r['ms_per_launch']) if rooflines else None
    out = {
        'metric': METRIC,
        'value': round(value, 3),
        'unit': 'V-cycle applies/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms_per_step, 4),
        'higher_is_better': True,
        'scaling': 'strong',
        'vs_baseline': None,
        'dtype': 'f64',
        'data': 'synthetic (P1 bidomain matrix generated in-library; r = uniform(-1,1), seed 1234)',
        'config': {
            'workload': '%s_%dd nrefs=%d gamma=%g metric_mono (profile %s)'
                        % (args.problem, args.dim, args.nrefs, args.gamma, PROFILE_NAMES[args.smoother]
                           + (', W-cycle' if args.cycle == 'W' else '') + (', coarse scaling' if args.scaling else '')),
            'n': n, 'N': sysm.N, 'nnz': sysm.nnz, 'levels': levels,
            'parallelism': 'single' if world == 1 else 'row-partition x%d (%s halo)' % (
                world, 'host-staged gloo' if gloo else 'RCCL'),
            'device_layout': layout,
        },
        'hbm_GBps_alg': round(apply_bytes / 1e9 / (ms_per_step * 1e-3), 1),
        'apply_GB_alg': round(apply_bytes / 1e9, 4),
        'graph_ms_per_step': graph_ms,
        'dist_graph': graph_info,
        'roofline': roofline,
        'roofline_kernels': rooflines,
        'level0_format': fmt0,
        'k_region': kregion,
        'cpu_baseline': cpu,
        'setup': dict(setup_info, generate_s=round(t_gen, 2)),
        'breakdown': breakdown,
        'pcg': pcg,
        'check_1gpu': check_1gpu,
        'pcg_profiles': profiles,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    B.close()
    if H is not None:
        H.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
