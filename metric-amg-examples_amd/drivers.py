"""Problem drivers: the reference's command lines on this framework.

    python -m metric_amg_examples_amd.drivers bidomain_3d -nrefs 6 -gamma 1e6 -precond metric_mono
    python -m metric_amg_examples_amd.drivers emi_3d -nrefs 5 -gamma 1e6 -precond metric
    python -m metric_amg_examples_amd.drivers emi_3d1d -gamma 1e4 -radius 1.0 -dump 1 -outdir D/
    python -m metric_amg_examples_amd.drivers run_solver_3d1d -infile input_metric.dat -indir D/ -outdir O/
    torchrun --nproc-per-node 8 -m metric_amg_examples_amd.drivers emi_3d1d_sweep -n 48

Each mirrors a reference script's CLI and output:
  bidomain_2d / bidomain_3d   src/bidomain_2d.py:105-278, src/bidomain_3d.py:52-220
  emi_2d / emi_3d             src/emi_2d.py:133-263, src/emi_3d.py:60-196
  emi_3d1d                    src/emi_3d1d.py:99-167 (dump / solve)
  run_solver_3d1d             src/run_solver_3d1d.py:17-38 (HAZmath file-based solve)
  emi_3d1d_sweep              run_emi_3d1d.sh:5-17 (radius x gamma loop), its
                              independent solves sharded over the ranks
Mesh loops: n = 2^i for i in [5, 5+nrefs) (bidomain 2-D), [3, 3+nrefs)
(bidomain 3-D), [6, 6+nrefs) (EMI 2-D), [2, 2+nrefs) (EMI 3-D).  Every solve
appends the reference's iters row ``ndofs niters cond timeKSP r h``
(src/bidomain_2d.py:149,259) to results/<problem>/iters_<...>.txt; timeKSP
spans preconditioner setup + CG, as in the reference (:176-197).
The bidomain and EMI drivers solve against the reference's manufactured
solutions (csrc/mms.cpp, mms.py; src/bidomain_2d.py:7-99, src/emi_2d.py:8-128)
and append the error row
``ndofs h |eu1|_1 r|eu1|_1 |eu2|_1 r|eu2|_1`` (H1 errors and rates,
src/bidomain_2d.py:150,239-270) to results/<problem>/error_<...>.txt;
``-rhs random`` uses the bench's seeded uniform(-1,1) vector instead.
``-profile reference`` (default) takes the AMG parameters the reference's
driver takes (metric_mono: parameters_metric_schwarz; metric / amg: the
factories' default dicts); ``-profile mi355x`` the GPU profile
(parameters_metric_mi355x) for every -precond choice.
Differences (stated, not hidden): the matrices come from the in-library
generators (problems.py; FEniCS is absent); the EMI drivers' manufactured
solutions are restated in mms.py (src/emi_2d.py:8-128); the 3D-1D neuron mesh
is the synthetic ``problems.neuron_curve``.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

from . import fileio, mms, parameters as P, problems
from .amg import MetricAMG
from .krylov import ConjGrad
from .precond import (get_block_diag_precond, get_hazmath_amg_precond, get_hazmath_metric_precond,
                      get_hazmath_metric_precond_mono, solve_haznics)

HEADERS_KSP = ['ndofs', 'niters', 'cond', 'timeKSP', 'r', 'h']
HEADERS_ERROR = ['ndofs', 'h', '|eu1|_1', 'r|eu1|_1', '|eu2|_1', 'r|eu2|_1']


def _iters_path(result_dir, precond, what='iters', **kv):
    tail = '_'.join('%s%s' % (k, v) for k, v in kv.items())
    return os.path.join(result_dir, '%s_precond%s_%s.txt' % (what, precond, tail))


def _append(path, row, first, headers=HEADERS_KSP):
    with open(path, 'w' if first else 'a') as out:
        if first:
            out.write('%s\n' % ' '.join(headers))
        out.write('%s\n' % ' '.join(map(str, row)))


def _profile_params(profile, precond):
    """The parameter dict of a -precond choice: 'reference' = the dict the
    reference's driver passes (src/bidomain_3d.py:138-147: metric_mono ->
    parameters_metric_schwarz; 'metric' and 'amg' call the factories without
    parameters, i.e. their defaults, src/utils.py:20-38,60-82), 'mi355x' =
    the GPU profile (parameters_metric_mi355x, nodal SA V-cycle, node-block
    Jacobi) for every choice."""
    if profile == 'mi355x':
        return P.parameters_metric_mi355x
    if precond in ('metric_mono', 'metric_hazmath'):
        return P.parameters_metric_schwarz
    return None


def _solve(A, W, b, precond, idofs, tol, maxiter, monolithic_params=None):
    """setup + CG, timed together (the reference's timeKSP)."""
    then = time.time()
    Asp = A.scipy() if hasattr(A, 'scipy') else A
    nf = 2 if W[0] == W[1] else 1
    if precond == 'metric_mono':
        BB = get_hazmath_metric_precond_mono(A, W, parameters=monolithic_params, interface_dofs=idofs,
                                             num_functions=nf)
        Aop = A                              # same object: device-resident PCG
    elif precond == 'metric':
        BB = get_hazmath_metric_precond(Asp, W, parameters=monolithic_params, interface_dofs=idofs,
                                        num_functions=nf)
        Aop = BB.Aop
    elif precond == 'amg':
        BB = get_hazmath_amg_precond(Asp, W, parameters=monolithic_params)
        Aop = BB._Aop
    elif precond == 'diag':
        BB = get_block_diag_precond(Asp, W)
        Aop = Asp
    else:
        raise ValueError(precond)
    solver = ConjGrad(Aop, precond=BB, tolerance=tol, maxiter=maxiter)
    x = solver * b
    dt = time.time() - then
    niters = len(solver.residuals) - 1
    eigs = solver.eigenvalue_estimates()
    cond = float(max(eigs) / min(eigs))
    return x, niters, cond, dt, solver.residuals[-1], BB


def bidomain(argv, dim):
    ap = argparse.ArgumentParser(prog='bidomain_%dd' % dim)
    ap.add_argument('-nrefs', type=int, default=1)
    ap.add_argument('-kappa1', type=float, default=2)
    ap.add_argument('-kappa2', type=float, default=3)
    ap.add_argument('-gamma', type=float, default=1)
    ap.add_argument('-pdegree', type=int, default=1, choices=(1,))
    ap.add_argument('-precond', type=str, default='metric_mono',
                    choices=('metric_mono', 'metric', 'amg', 'diag', 'metric_hazmath'))
    ap.add_argument('-save', type=int, default=0)
    ap.add_argument('-results', type=str, default='./results')
    ap.add_argument('-rhs', type=str, default='mms', choices=('mms', 'random'))
    ap.add_argument('-profile', type=str, default='reference', choices=('reference', 'mi355x'),
                    help="AMG parameters: the reference driver's dicts, or the GPU profile")
    args, _ = ap.parse_known_args(argv)
    prm = _profile_params(args.profile, args.precond)
    rdir = os.path.join(args.results, 'bidomain_%dd' % dim)
    os.makedirs(rdir, exist_ok=True)
    tags = dict(kappa1=args.kappa1, kappa2=args.kappa2, gamma=args.gamma, pdegree=args.pdegree)
    path = _iters_path(rdir, args.precond, **tags)
    epath = _iters_path(rdir, args.precond, 'error', **tags)
    i0 = 5 if dim == 2 else 3
    rows = []
    errors0 = h0 = None
    for k, n in enumerate(2 ** i for i in range(i0, i0 + args.nrefs)):
        s = problems.bidomain(dim, n, args.gamma, args.kappa1, args.kappa2)
        if args.rhs == 'mms':
            b = problems.bidomain_mms_rhs(dim, n, args.gamma, args.kappa1, args.kappa2)
        else:
            b = problems.seeded_rhs(s.N)
        if args.precond == 'metric_hazmath':     # the whole solve in the library (src/bidomain_2d.py:181-186)
            niters, xb, dt = solve_haznics(s, b, s.W, interface_dofs=s.idofs, parameters=prm)
            x, cond, r = np.concatenate(xb), -1, 0
        else:
            x, niters, cond, dt, r, _ = _solve(s, s.W, b, args.precond, s.idofs, 1e-8, 500, prm)
        h = np.sqrt(dim) / n            # dolfin hmin: the simplices' longest edge
        row = (s.N, niters, cond, dt, r, h)
        rows.append(row)
        _append(path, row, k == 0)
        print('bidomain_%dd n=%d ndofs=%d niters=%d cond=%.3g timeKSP=%.3fs r=%.3e'
              % (dim, n, s.N, niters, cond, dt, r), flush=True)
        if args.rhs != 'mms':
            continue
        xs = x.cpu().numpy() if hasattr(x, 'cpu') else np.asarray(x)
        errors = np.array(problems.bidomain_mms_errors(dim, n, xs, args.gamma, args.kappa1, args.kappa2))
        rates = [np.nan] * 2 if errors0 is None else np.log(errors / errors0) / np.log(h / h0)
        errors0, h0 = errors, h
        erow = (s.N, h) + tuple(v for pair in zip(errors, rates) for v in pair)
        _append(epath, erow, k == 0, HEADERS_ERROR)
        print('    |eu1|_1=%.4e (rate %.3f)  |eu2|_1=%.4e (rate %.3f)'
              % (errors[0], rates[0], errors[1], rates[1]), flush=True)
    return rows


def emi(argv, dim):
    ap = argparse.ArgumentParser(prog='emi_%dd' % dim)
    ap.add_argument('-nrefs', type=int, default=1)
    ap.add_argument('-kappa1', type=float, default=2)
    ap.add_argument('-kappa2', type=float, default=3)
    ap.add_argument('-gamma', type=float, default=5)
    ap.add_argument('-pdegree', type=int, default=1, choices=(1,))
    ap.add_argument('-precond', type=str, default='metric', choices=('metric', 'metric_mono', 'diag'))
    ap.add_argument('-save', type=int, default=0)
    ap.add_argument('-results', type=str, default='./results')
    ap.add_argument('-rhs', type=str, default='mms', choices=('mms', 'random'))
    ap.add_argument('-profile', type=str, default='reference', choices=('reference', 'mi355x'),
                    help="AMG parameters: the reference's default dict (src/utils.py:60-82), or the GPU profile")
    args, _ = ap.parse_known_args(argv)
    prm = _profile_params(args.profile, args.precond)
    rdir = os.path.join(args.results, 'emi_%dd' % dim)
    os.makedirs(rdir, exist_ok=True)
    tags = dict(kappa1=args.kappa1, kappa2=args.kappa2, gamma=args.gamma, pdegree=args.pdegree)
    path = _iters_path(rdir, args.precond, **tags)
    epath = _iters_path(rdir, args.precond, 'error', **tags)
    i0 = 6 if dim == 2 else 2
    rows = []
    errors0 = h0 = None
    for k, n in enumerate(2 ** i for i in range(i0, i0 + args.nrefs)):
        s = problems.emi(dim, n, args.gamma, args.kappa1, args.kappa2)
        if args.rhs == 'mms':
            b = mms.emi_mms_rhs(dim, n, args.gamma, args.kappa1, args.kappa2)
        else:
            b = [problems.seeded_rhs(s.W[0], 1234), problems.seeded_rhs(s.W[1], 4321)]
        then = time.time()
        if args.precond == 'diag':
            BB = get_block_diag_precond(s.blocks, s.W)
        else:
            BB = get_hazmath_metric_precond(s.blocks, s.W, parameters=prm, interface_dofs=s.idofs,
                                            num_functions=2)
        solver = ConjGrad(s, precond=BB, tolerance=1e-10, maxiter=500)   # src/emi_3d.py:143
        x = solver * b
        dt = time.time() - then
        niters = len(solver.residuals) - 1
        eigs = solver.eigenvalue_estimates()
        h = np.sqrt(dim) / n
        row = (s.N, niters, float(max(eigs) / min(eigs)), dt, solver.residuals[-1], h)
        rows.append(row)
        _append(path, row, k == 0)
        print('emi_%dd n=%d ndofs=%d niters=%d cond=%.3g timeKSP=%.3fs' % (dim, n, s.N, niters, row[2], dt),
              flush=True)
        if args.rhs != 'mms':
            continue
        xs = [xi.cpu().numpy() if hasattr(xi, 'cpu') else np.asarray(xi) for xi in x] \
            if isinstance(x, (list, tuple)) else (x.cpu().numpy() if hasattr(x, 'cpu') else np.asarray(x))
        errors = np.array(mms.emi_mms_errors(dim, n, xs, args.gamma, args.kappa1, args.kappa2))
        rates = [np.nan] * 2 if errors0 is None else np.log(errors / errors0) / np.log(h / h0)
        errors0, h0 = errors, h
        _append(epath, (s.N, h) + tuple(v for pair in zip(errors, rates) for v in pair), k == 0,
                HEADERS_ERROR)
        print('    |eu1|_1=%.4e (rate %.3f)  |eu2|_1=%.4e (rate %.3f)'
              % (errors[0], rates[0], errors[1], rates[1]), flush=True)
    return rows


def emi_3d1d(argv):
    ap = argparse.ArgumentParser(prog='emi_3d1d')
    ap.add_argument('-gamma', type=float, default=1)
    ap.add_argument('-dump', type=int, default=0, choices=(0, 1))
    ap.add_argument('-radius', type=float, default=1)
    ap.add_argument('-n', type=int, default=32, help='cells per direction of the tissue cube')
    ap.add_argument('-outdir', type=str, default='./data/emi_3d1d/')
    args, _ = ap.parse_known_args(argv)
    t0 = time.time()
    s = problems.emi_3d1d(args.n, args.gamma, args.radius)
    print('System setup and assembly time: %.3f' % (time.time() - t0), flush=True)
    A = s.scipy()
    b = problems.seeded_rhs(s.N)
    if args.dump:
        fileio.dump_system(A, b, s.W, args.outdir)
        return None
    # alternative solver: the file-free path of solve_haznics (src/utils.py:95-127)
    B = MetricAMG(A, s.W, idofs=s.idofs, parameters=P.parameters_metric_3d1d)
    solver = ConjGrad(A, precond=B, tolerance=1e-6, maxiter=1000, stop_type=1)
    solver * b
    print('niters %d' % (len(solver.residuals) - 1))
    return len(solver.residuals) - 1


def fenics_metric_solver_xd_1d(sfile: str, mdir: str, odir: str, quiet: bool = False) -> int:
    """HAZmath's file-based 3D-1D solve (haznics.fenics_metric_solver_xd_1d,
    called at src/run_solver_3d1d.py:38): parameters from the .dat file,
    A / b / idofs from mdir (utils.dump_system format), CG with the file's
    stopping rule, metric AMG seeded at the 1D dofs; writes odir/solution.txt.
    Returns the iteration count."""
    d = fileio.read_dat(sfile)
    params, solver_prm, notes = fileio.dat_to_parameters(d)
    A, b, idofs, idofs3d = fileio.load_system(mdir)
    N = A.shape[0]
    W = [N - len(idofs), len(idofs)] if idofs is not None else [N]
    t0 = time.time()
    B = MetricAMG(A, W, idofs=idofs, parameters=params)
    t1 = time.time()
    st = solver_prm['stop_type']
    cg = ConjGrad(A, precond=B, tolerance=solver_prm['tol'], maxiter=solver_prm['maxit'],
                  stop_type=1 if st == 1 else None, relativeconv=st == 2)
    x = cg * b
    t2 = time.time()
    os.makedirs(odir, exist_ok=True)
    fileio.write_solution(os.path.join(odir, 'solution.txt'), x)
    niters = len(cg.residuals) - 1
    if not quiet:
        for n in notes:
            print('[mamg] parameter substitution: %s' % n)
        rel = cg.residual_norms[-1] / max(np.linalg.norm(b), 1e-300)
        print('Number of iterations = %d, relative residual = %.6e' % (niters, rel))
        print('AMG setup (%s): %.3f s, solve: %.3f s, levels: %d'
              % (B.setup_path, t1 - t0, t2 - t1, B.num_levels), flush=True)
    return niters


def run_solver_3d1d(argv):
    ap = argparse.ArgumentParser(prog='run_solver_3d1d')
    ap.add_argument('-infile', type=str, default='./src/input_metric.dat')
    ap.add_argument('-indir', type=str, default='./data/emi_3d1d/')
    ap.add_argument('-outdir', type=str, default='./results/emi_3d1d/')
    args, _ = ap.parse_known_args(argv)
    if not os.path.exists(args.infile) or not os.path.exists(args.indir):
        raise SystemExit('input file or matrix directory missing')
    return fenics_metric_solver_xd_1d(os.path.abspath(args.infile), os.path.abspath(args.indir) + '/',
                                      os.path.abspath(args.outdir) + '/')


# ---- the 3D-1D sweep (BASELINE config 5) on N GPUs --------------------------
# run_emi_3d1d.sh:5-17 loops radius x gamma and runs one independent
# assemble -> setup -> PCG per pair.  Those solves are the sweep's units: on N
# GPUs every rank takes units k with k % N == rank (one process per GPU, no
# data-path collective; the 117 K-row system is far too small to row-partition
# profitably), and rank 0 gathers the rows (one all_gather_object over gloo at
# the end) and writes them in the script's loop order.
SWEEP_RADII = (0.0, 0.2, 1.0, 5.0)                      # run_emi_3d1d.sh:5
SWEEP_GAMMAS = (1e0, 1e2, 1e4, 1e6, 1e8, 1e10)          # run_emi_3d1d.sh:7
HEADERS_SWEEP = ['radius', 'gamma', 'ndofs', 'niters', 'timeKSP', 'relres', 'levels', 'rank']


def sweep_units(radii=SWEEP_RADII, gammas=SWEEP_GAMMAS):
    """(radius, gamma) pairs in the script's loop order (radius outer)."""
    return [(float(r), float(g)) for r in radii for g in gammas]


def shard_units(units, rank: int, world: int):
    """The units of one rank: (index, unit) for index % world == rank."""
    if not 0 <= rank < world:
        raise ValueError('rank %d outside world %d' % (rank, world))
    return [(k, u) for k, u in enumerate(units) if k % world == rank]


def solve_3d1d_unit(n: int, radius: float, gamma: float, params=None, device=None,
                    tol: float = 1e-6, maxiter: int = 1000) -> dict:
    """One unit of the sweep: assemble (problems.emi_3d1d), metric-AMG setup
    seeded at the 1D dofs, PCG stopped on ||r|| / ||b|| (the .dat file's
    stop type 1, src/input_metric.dat:54) -- src/emi_3d1d.py:99-167 with
    run_solver_3d1d's solve.  timeKSP = setup + PCG."""
    s = problems.emi_3d1d(n, gamma, radius)
    A = s.scipy()
    b = problems.seeded_rhs(s.N)
    t0 = time.time()
    kw = {} if device is None else dict(device=device)
    B = MetricAMG(A, s.W, idofs=s.idofs, parameters=params or P.parameters_metric_3d1d, **kw)
    cg = ConjGrad(A, precond=B, tolerance=tol, maxiter=maxiter, stop_type=1)
    x = cg * b
    dt = time.time() - t0
    xs = x.cpu().numpy() if hasattr(x, 'cpu') else np.asarray(x)
    rel = float(np.linalg.norm(b - A @ xs) / np.linalg.norm(b))
    row = dict(radius=radius, gamma=gamma, ndofs=int(s.N), niters=len(cg.residuals) - 1,
               timeKSP=round(dt, 4), relres=rel, levels=B.num_levels)
    B.close()
    return row


def run_sweep(units, solve, rank: int = 0, world: int = 1, gather=None):
    """Solve this rank's shard of `units` with solve(unit) -> dict, then
    gather every rank's rows (gather(obj) -> list over ranks, e.g.
    torch.distributed.all_gather_object).  Returns (rows in unit order,
    this rank's wall seconds, the max over ranks)."""
    t0 = time.time()
    mine = []
    for k, u in shard_units(units, rank, world):
        row = dict(solve(u))
        row['rank'] = rank
        mine.append((k, row))
    wall = time.time() - t0
    parts = [(mine, wall)] if gather is None else gather((mine, wall))
    rows = sorted((kr for part, _ in parts for kr in part), key=lambda kr: kr[0])
    if [k for k, _ in rows] != list(range(len(units))):
        raise RuntimeError('sweep gather lost or duplicated units: %s' % [k for k, _ in rows])
    return [r for _, r in rows], wall, max(w for _, w in parts)


def emi_3d1d_sweep(argv):
    ap = argparse.ArgumentParser(prog='emi_3d1d_sweep')
    ap.add_argument('-n', type=int, default=48, help='cells per direction of the tissue cube')
    ap.add_argument('-radii', type=str, default=','.join(map(str, SWEEP_RADII)))
    ap.add_argument('-gammas', type=str, default=','.join('%g' % g for g in SWEEP_GAMMAS))
    ap.add_argument('-results', type=str, default='./results')
    args, _ = ap.parse_known_args(argv)
    import json
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    gather = None
    device = None
    import torch
    if torch.cuda.is_available():
        device = local % torch.cuda.device_count()
        torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('gloo')   # one gather of the result rows at the end

        def gather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out
    units = sweep_units([float(v) for v in args.radii.split(',')], [float(v) for v in args.gammas.split(',')])
    rows, _, wall = run_sweep(units, lambda u: solve_3d1d_unit(args.n, u[0], u[1], device=device),
                              rank, world, gather)
    if rank == 0:
        rdir = os.path.join(args.results, 'emi_3d1d')
        os.makedirs(rdir, exist_ok=True)
        path = os.path.join(rdir, 'iters_sweep_n%d.txt' % args.n)
        for k, r in enumerate(rows):
            _append(path, [r[h] for h in HEADERS_SWEEP], k == 0, HEADERS_SWEEP)
            print('emi_3d1d radius=%g gamma=%g ndofs=%d niters=%d timeKSP=%.3fs relres=%.2e (rank %d)'
                  % (r['radius'], r['gamma'], r['ndofs'], r['niters'], r['timeKSP'], r['relres'], r['rank']),
                  flush=True)
        print(json.dumps({'sweep': 'emi_3d1d', 'n': args.n, 'units': len(units), 'ranks': world,
                          'wall_s': round(wall, 3), 'solves_per_s': round(len(units) / wall, 3),
                          'niters': [r['niters'] for r in rows]}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    return rows


COMMANDS = {
    'bidomain_2d': lambda a: bidomain(a, 2),
    'bidomain_3d': lambda a: bidomain(a, 3),
    'emi_2d': lambda a: emi(a, 2),
    'emi_3d': lambda a: emi(a, 3),
    'emi_3d1d': emi_3d1d,
    'run_solver_3d1d': run_solver_3d1d,
    'emi_3d1d_sweep': emi_3d1d_sweep,
}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in COMMANDS:
        print(__doc__)
        return 2
    COMMANDS[argv[0]](argv[1:])
    return 0


if __name__ == '__main__':
    sys.exit(main())
