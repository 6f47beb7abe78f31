#!/usr/bin/env python3
"""Full-size rehearsal of the N-rank path on one GPU (virtual ranks).

    python bench/dist_rehearsal.py [--nrefs 6] [--ranks 8] [--source device|host]

Builds the P rank-local handles of bidomain_3d (each runs the same
deterministic setup as a real rank would, then keeps its rows), reports per
rank the setup wall time, device bytes held and the process's peak host RSS,
then runs one virtual distributed apply (device copies stand in for RCCL,
same counts/offsets) and compares it with the single-GPU apply.  This is what
each process of `bench.py --gpus P` does before its timed region.

--source device (default, as bench.py --gpus P): A_0 is generated in HBM by
the gfx950 generator (problems.bidomain_device) and every rank's setup reads
it there, so the host holds only sizes, seeds and the rank's plan; the
per-rank RSS reported is the process's RSS growth over that rank's setup
(< 4 GB).  --source host: the global host CSR, as
in round 3.  --check-host additionally builds the host-source handles and
checks the two virtual applies bitwise.

With MAMG_DIST_TEST=dry it instead times each rank's cycle with the exchanges
skipped: the compute part of the P-GPU apply (RCCL latency not included),
eager and as hipGraph replays.
"""
import argparse
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rss_gb():
    """current resident set of this process (GB)"""
    with open('/proc/self/statm') as f:
        return int(f.read().split()[1]) * os.sysconf('SC_PAGE_SIZE') / 2**30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nrefs', type=int, default=6)
    ap.add_argument('--gamma', type=float, default=1e6)
    ap.add_argument('--ranks', type=int, default=8)
    ap.add_argument('--source', choices=('device', 'host'), default='device')
    ap.add_argument('--check-host', action='store_true')
    ap.add_argument('--profile', choices=('mi355x', 'schwarz', 'patch'), default='mi355x',
                    help='mi355x: the GPU profile (default); schwarz: the reference preset '
                         'parameters_metric_schwarz verbatim (node patches on level 0); patch: '
                         'parameters_metric_mi355x_patch')
    args = ap.parse_args()
    import numpy as np
    import torch
    import metric_amg_examples_amd as M
    n = M.problems.finest_n(3, args.nrefs)
    for name in ('MAMG_DIST_TEST', 'MAMG_K_COL16'):   # the library reads no environment: pass them on
        if os.environ.get(name):
            M._lib.set_option(name, os.environ[name])
    torch.cuda.init()
    rss_start = rss_gb()
    if args.source == 'device':
        A = M.problems.bidomain_device(3, n, args.gamma)
        s = M.problems.bidomain_meta(3, n, A[1].numel())
    else:
        s = M.problems.bidomain(3, n, args.gamma)
        A = s
    r = M.problems.seeded_rhs(s.N)
    prm = {'mi355x': None, 'schwarz': M.parameters.parameters_metric_schwarz,
           'patch': M.parameters.parameters_metric_mi355x_patch}[args.profile]
    out = {'N': s.N, 'ranks': args.ranks, 'source': args.source, 'profile': args.profile,
           'rss_start_GB': round(rss_start, 2),
           'rss_after_A0_GB': round(rss_gb(), 2), 'per_rank': []}
    hs = []
    for p in range(args.ranks):
        torch.cuda.synchronize()
        m0 = torch.cuda.mem_get_info()[0]
        r0 = rss_gb()
        t0 = time.time()
        hs.append(M.DistMetricAMG(A, s.W, idofs=s.idofs, rank=p, nranks=args.ranks, comm_id=None,
                                  parameters=prm, num_functions=2, print_level=2))
        torch.cuda.synchronize()
        t = time.time() - t0
        held = m0 - torch.cuda.mem_get_info()[0]
        r1 = rss_gb()
        peak = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20
        # a real rank = the process start + A_0 (on the host only with
        # --source host) + its own setup; the growth over this rank's setup
        # is what the handle keeps plus what the setup left in the allocator
        out['per_rank'].append({'rank': p, 'setup_s': round(t, 2), 'device_GB': round(held / 1e9, 2),
                                'rss_growth_GB': round(r1 - r0, 2), 'process_peak_rss_GB': round(peak, 2),
                                'nodes': [hs[-1].o0, hs[-1].o1],
                                'apply_launches': hs[-1].apply_launches})
        print('rank %d: setup %.1fs, device %.2f GB, RSS +%.2f GB (now %.2f, peak %.2f)'
              % (p, t, held / 1e9, r1 - r0, r1, peak), flush=True)
    out['rank_rss_estimate_GB'] = round(out['rss_after_A0_GB'] + max(q['rss_growth_GB'] for q in out['per_rank']), 2)
    rs = [torch.as_tensor(h.local_slice(r)).cuda() for h in hs]
    zs = [torch.zeros_like(x) for x in rs]
    if os.environ.get('MAMG_DIST_TEST') == 'dry':
        # compute-only time of each rank's cycle (exchanges skipped; the
        # numbers exclude RCCL latency, the results are not used)
        names = ['L0_resid', 'L0_smooth_spmv', 'L0_smoother', 'L0_restrict', 'L0_prolong',
                 'coarse_levels', 'coarsest_dense', 'misc', 'comm']
        for p, h in enumerate(hs):
            h.time_apply(rs[p], zs[p], 3, 0)
            ms, _, _ = h.time_apply(rs[p], zs[p], 20, 0)
            ms1, kms, _ = h.time_apply(rs[p], zs[p], 5, 1)
            try:
                h.time_apply(rs[p], zs[p], 3, 2)          # hipGraph replays (captured once)
                msg, _, _ = h.time_apply(rs[p], zs[p], 20, 2)
            except M._lib.MamgError:                      # too many ops for one graph
                msg = float('nan')
            out['per_rank'][p]['compute_ms_per_apply'] = round(ms, 4)
            out['per_rank'][p]['compute_ms_per_apply_graph'] = round(msg, 4)
            out['per_rank'][p]['classes_ms'] = {k: round(v, 4) for k, v in zip(names, kms) if v}
            print('rank %d: compute-only %.3f ms/apply eager, %.3f graph %s' % (p, ms, msg, out['per_rank'][p]['classes_ms']),
                  flush=True)
        print(json.dumps(out), flush=True)
        return
    M.DistMetricAMG.virtual_apply(hs, rs, zs)
    zg = [torch.full_like(x, float('nan')) for x in rs]
    try:
        M.DistMetricAMG.virtual_apply(hs, rs, zg, graph=True)      # the lockstep apply as one hipGraph
        torch.cuda.synchronize()
        out['graph_equals_eager_bitwise'] = all(bool(torch.equal(a, b)) for a, b in zip(zs, zg))
    except M._lib.MamgError as e:          # too many ops for one graph: eager only
        out['graph'] = str(e)
    del zg
    nv = s.N // 2

    def gather(hs, zs):
        z = np.zeros(s.N)
        for h, zz in zip(hs, zs):
            zz = zz.cpu().numpy()
            k = h.o1 - h.o0
            z[h.o0:h.o1] = zz[:k]
            z[nv + h.o0:nv + h.o1] = zz[k:]
        return z

    z = gather(hs, zs)
    for h in hs:
        h.close()
    if args.check_host and args.source == 'device':
        sh = M.problems.bidomain(3, n, args.gamma)
        hh = [M.DistMetricAMG(sh, sh.W, idofs=sh.idofs, rank=p, nranks=args.ranks, comm_id=None,
                              num_functions=2) for p in range(args.ranks)]
        zh = [torch.zeros_like(x) for x in rs]
        M.DistMetricAMG.virtual_apply(hh, rs, zh)
        torch.cuda.synchronize()
        out['device_vs_host_source_max_abs'] = float(np.max(np.abs(gather(hh, zh) - z)))
        for h in hh:
            h.close()
        del sh
    B = M.MetricAMG(A, s.W, idofs=s.idofs, parameters=prm, num_functions=2, setup='gpu')
    z1 = B * r
    if args.profile != 'mi355x':      # the one-GPU apply's time, for the per-rank compute comparison
        import torch as _t
        rt = _t.as_tensor(r).cuda()
        zt = _t.zeros_like(rt)
        out['single_gpu_ms_per_apply'] = round(B.time_apply(rt, zt, 3, 0)[0], 3)
    out['rel_diff_vs_single_gpu'] = float(np.linalg.norm(z - z1) / np.linalg.norm(z1))
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
