"""Diagnosis of an intermittent wrong apply seen once in
tests/test_gpu.py::test_k_kernel_variants (a MAMG_REHOME=0 handle built while
two others are alive): the test's handle sequence repeated, each apply
compared with the oracle, with HBM freed by torch poisoned (0xff bytes = NaN)
before every setup so that a read of uninitialised device memory shows.
Usage: python bench/kflake.py ITERS [poison_MiB]"""
import os
import sys

sys.path.insert(0, '.')
sys.path.insert(0, 'oracle')
import numpy as np
import torch

import mamg_oracle as mo
import metric_amg_examples_amd as M

os.environ['MAMG_SELL_MIN_ROWS'] = '1'
s = M.problems.bidomain(3, 16, 1e6)
A = s.scipy()
rn = mo.seeded_rhs(s.N)
r = torch.as_tensor(rn).cuda()
zo = mo.setup(A, mo.Params(num_functions=2), idofs=s.idofs).apply(rn)
poison_mib = int(sys.argv[2]) if len(sys.argv) > 2 else 2048


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def poison():
    if poison_mib <= 0:
        return
    t = torch.full((poison_mib << 20,), 0xff, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    del t
    torch.cuda.empty_cache()


def err(z):
    torch.cuda.synchronize()
    return rel(z.cpu().numpy(), zo)


nbad = 0
for it in range(int(sys.argv[1])):
    for variant in ('0', '1', '2'):
        out = []
        os.environ.pop('MAMG_REHOME', None)
        os.environ.pop('MAMG_K_LAYOUT', None)
        os.environ['MAMG_K_VARIANT'] = '1'
        poison()
        B1 = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        out.append(('B1', err(B1.matvec(r))))
        os.environ['MAMG_K_VARIANT'] = variant
        poison()
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        out.append(('B', err(B.matvec(r))))
        zz = torch.empty_like(r)
        for lay in ('split', 'block'):
            os.environ['MAMG_K_LAYOUT'] = lay
            B.time_apply(r, zz, 1, 0)
        os.environ.pop('MAMG_K_LAYOUT', None)
        B.time_apply(r, zz, 1, 0)
        out.append(('B relayout', err(zz)))
        os.environ['MAMG_REHOME'] = '0'
        poison()
        B0 = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2)
        out.append(('B0', err(B0.matvec(r))))
        out.append(('B again', err(B.matvec(r))))
        out.append(('B1 again', err(B1.matvec(r))))
        bad = max(e for _, e in out) > 1e-10
        nbad += bad
        print(it, 'variant', variant, ' '.join('%s %.1e' % kv for kv in out), 'BAD' if bad else '', flush=True)
        for b in (B, B0, B1):
            b.close()
print('bad', nbad, flush=True)
