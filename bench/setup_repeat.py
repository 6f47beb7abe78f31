"""Determinism of the GPU setup and of the apply: the same problem set up
ITERS times on the GPU (mamg_gpu_host_setup, levels exported) and compared
bitwise with the first setup level by level, and the apply B r of handles
built with MAMG_HALF 1 / 0 compared bitwise across repetitions.  Prints the
first differing array of each repetition.
Usage: python bench/setup_repeat.py ITERS [churn]"""
import os
import sys

sys.path.insert(0, '.')
sys.path.insert(0, 'oracle')
import numpy as np

import mamg_oracle as mo
import metric_amg_examples_amd as M

os.environ['MAMG_SELL_MIN_ROWS'] = '1'
iters = int(sys.argv[1])
churn = len(sys.argv) > 2 and sys.argv[2] == 'churn'


def churn_memory():
    """a larger handle set up, solved with and closed: HBM the next setup
    reuses then holds finite, nonzero data (as in the test suite)"""
    if not churn:
        return
    import torch
    t = torch.rand(1 << 27, dtype=torch.float64, device='cuda') * 1e3 + 1.0
    torch.cuda.synchronize()
    del t
    torch.cuda.empty_cache()
    sb = M.problems.bidomain(3, 24, 1e6)
    Ab = sb.scipy()
    Bb = M.MetricAMG(Ab, sb.W, idofs=sb.idofs, num_functions=2)
    M.ConjGrad(Ab, precond=Bb, tolerance=1e-8, maxiter=50) * mo.seeded_rhs(sb.N)
    Bb.close()


def levels(H):
    out = []
    for l in range(H.num_levels):
        d = H.level(l)
        for k in sorted(d):
            v = d[k]
            if isinstance(v, tuple):
                out += [('%d.%s.%d' % (l, k, i), a) for i, a in enumerate(v[:3])]
            elif isinstance(v, np.ndarray):
                out.append(('%d.%s' % (l, k), v))
    return out


def first_diff(a, b):
    if len(a) != len(b):
        return 'levels %d vs %d' % (len(a) // 10, len(b) // 10)
    for (ka, va), (kb, vb) in zip(a, b):
        if ka != kb or va.shape != vb.shape or not np.array_equal(va, vb):
            return '%s differs (%s vs %s)' % (ka, va.shape, vb.shape)
    return None


nbad = 0
for dim, n, g, kw in ((3, 16, 1e4, dict(post_fusion=0)), (3, 16, 1e6, dict())):
    s = M.problems.bidomain(dim, n, g)
    A = s.scipy()
    r = mo.seeded_rhs(s.N)
    ref = levels(M.HostHierarchy(A, idofs=s.idofs, gpu=True, num_functions=2, **kw))
    host = levels(M.HostHierarchy(A, idofs=s.idofs, gpu=False, num_functions=2, **kw))
    print(dim, n, g, 'gpu setup vs host setup:', first_diff(ref, host) or 'bitwise', flush=True)
    z_ref = None
    for it in range(iters):
        d = first_diff(ref, levels(M.HostHierarchy(A, idofs=s.idofs, gpu=True, num_functions=2, **kw)))
        zs = []
        for half in ('1', '0'):
            churn_memory()
            os.environ['MAMG_HALF'] = half
            B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, **kw)
            zs.append(B * r)
            B.close()
        z_ref = zs[0] if z_ref is None else z_ref
        za = [np.array_equal(z, z_ref) for z in zs]
        bad = d is not None or not all(za)
        nbad += bad
        if bad or it % 10 == 0:
            print(it, 'setup', d or 'bitwise', 'apply half1/half0 = first:', za, 'BAD' if bad else '', flush=True)
    os.environ.pop('MAMG_HALF', None)
print('bad', nbad, flush=True)
