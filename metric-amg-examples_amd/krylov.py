"""ConjGrad with cbc.block semantics, driving the GPU preconditioner.

Reference use (/root/reference/src/bidomain_3d.py:149-160):
    AAinv = ConjGrad(AA_, precond=BB, tolerance=1E-8, show=4, maxiter=500,
                     callback=cbk)
    xx = AAinv * bb_
    niters = len(AAinv.residuals) - 1
    r_norm = AAinv.residuals[-1]
    eigenvalues = AAinv.eigenvalue_estimates()
cbc.block ``cgN`` [ext, recalled]: residuals are sqrt(<r, B r>), the
tolerance is absolute unless relativeconv, x0 = 0 unless initial_guess,
breakdown when <r, B r> < 0 (x restored) or <d, A d> == 0.

When ``precond`` is a MetricAMG built on the same operator and no callback
is given, the whole loop runs device-resident (``mamg_pcg_device``: level-0
SpMV, fused CG vector kernels, deterministic dots, hipGraph V-cycle);
otherwise the loop runs on the host with one ``B * r`` per iteration through
the C-ABI, exactly like the reference's cbc.block loop.
"""
from __future__ import annotations

import ctypes as C
import warnings

import numpy as np

from . import _lib
from .amg import MetricAMG


def lanczos_eigenvalues(alphas, betas):
    """Eigenvalues of the CG Lanczos tridiagonal (cbc.block
    eigenvalue_estimates): T00 = 1/a0, Tkk = 1/ak + b(k-1)/a(k-1),
    T(k,k-1) = sqrt(b(k-1))/a(k-1)."""
    n = len(alphas)
    if n == 0:
        return np.array([1.0])
    T = np.zeros((n, n))
    T[0, 0] = 1.0 / alphas[0]
    for k in range(1, n):
        T[k, k] = 1.0 / alphas[k] + betas[k - 1] / alphas[k - 1]
        T[k, k - 1] = np.sqrt(betas[k - 1]) / alphas[k - 1]
        T[k - 1, k] = T[k, k - 1]
    return np.sort(np.linalg.eigvalsh(T))


class ConjGrad:
    def __init__(self, A, precond=None, tolerance=1e-5, initial_guess=None, maxiter=200,
                 show=1, callback=None, relativeconv=False, device=None, stop_type=None, **kwargs):
        # block systems (src/emi_3d.py:143: CG on the 2x2 block matrix with
        # precond R^T Minv R): solved on the monolithic storage, where
        # R^T Minv R is Minv itself; block vectors in and out
        self._block_sizes = None
        if hasattr(A, 'blocks') or isinstance(A, (list, tuple)):
            from .precond import to_monolithic
            Am = getattr(precond, 'Aop', None)
            self._block_sizes = ([int(w) for w in A.W] if hasattr(A, 'W')
                                 else [blk[0].shape[0] for blk in A])
            A = Am if Am is not None else to_monolithic(A)
        if getattr(precond, 'monolithic', None) is not None:
            precond = precond.monolithic
        self.A = A
        self.B = precond
        self.tolerance = float(tolerance)
        self.initial_guess = initial_guess
        self.maxiter = int(maxiter)
        self.show = show
        self.callback = callback
        self.relativeconv = bool(relativeconv)
        self.device = device
        # stop_type None: cbc.block (sqrt(<r,Br>) vs tolerance); 1: HAZmath
        # linear_stop_type 1, ||r||_2 <= tolerance ||b||_2 (src/input_metric.dat:54)
        if stop_type not in (None, 1):
            raise ValueError('stop_type must be None (cbc.block) or 1 (||r||/||b||)')
        self.stop_type = stop_type
        self.residuals, self.alphas, self.betas = [], [], []
        self.residual_norms = []
        self.breakdown = False

    # ------------------------------------------------------------------
    def _device_ok(self):
        if self.device is False or self.callback is not None or self.stop_type is not None:
            return False
        B = self.B
        return isinstance(B, MetricAMG) and B._Aop is self.A

    def __mul__(self, b):
        if hasattr(b, 'data_ptr') and getattr(b, 'is_cuda', False):   # torch tensor in HBM
            return self.solve_device(b)
        blocks = isinstance(b, (list, tuple))
        if blocks:
            b = np.concatenate([np.asarray(bi, dtype=np.float64) for bi in b])
        if self.device is True and not self._device_ok():
            raise ValueError('ConjGrad(device=True) needs precond = a MetricAMG built on this A (the '
                             'device PCG uses its level-0 operator), no callback and the cbc.block stopping rule')
        if self._device_ok():
            x = self._solve_device(b)
        else:
            x = self._solve_host(b)
        if blocks:
            sizes = self._block_sizes or [len(x)]
            off = np.concatenate([[0], np.cumsum(sizes)])
            return [x[off[i]:off[i + 1]] for i in range(len(sizes))]
        return x

    def _solve_device(self, b):
        import torch
        bt = torch.as_tensor(np.ascontiguousarray(b, dtype=np.float64)).cuda()
        xt = self.solve_device(bt)
        torch.cuda.synchronize()
        return xt.cpu().numpy()

    def solve_device(self, bt, xt=None):
        """Device-resident solve: b (and x0 / the result) are float64 torch
        tensors in HBM; runs on torch's current stream, returns x (no host
        copies of the vectors; the residual history comes back to the host)."""
        import torch
        if not self._device_ok():
            raise ValueError('device solve needs precond = a MetricAMG built on this A, no callback and '
                             'the cbc.block stopping rule')
        B = self.B
        n = B.shape[0]
        if bt.dtype != torch.float64 or bt.numel() != n or not bt.is_contiguous():
            raise ValueError('b must be a contiguous float64 tensor of length %d' % n)
        if xt is None:
            if self.initial_guess is None:
                xt = torch.zeros_like(bt)
            else:
                xt = torch.as_tensor(np.ascontiguousarray(self.initial_guess, np.float64)).to(bt.device)
        res = np.zeros(self.maxiter + 1)
        al = np.zeros(max(self.maxiter, 1))
        be = np.zeros(max(self.maxiter, 1))
        it = C.c_int(0)
        stream = torch.cuda.current_stream()
        rc = B._L.mamg_pcg_device(B.handle, C.c_void_p(bt.data_ptr()), C.c_void_p(xt.data_ptr()),
                                  self.tolerance, self.maxiter, int(self.relativeconv),
                                  _lib.ptr(res, C.c_double), _lib.ptr(al, C.c_double),
                                  _lib.ptr(be, C.c_double), C.byref(it),
                                  C.c_void_p(stream.cuda_stream))
        k = it.value
        if rc == _lib.ERR_BREAKDOWN:
            self.breakdown = True
            msg = B._L.mamg_last_error().decode()
            if '<d,Ad> = 0' not in msg:        # the host loop stops silently on <d,Ad> = 0 too
                warnings.warn('ConjGrad breakdown: ' + msg)
            if k == 0 and res[0] == 0.0:
                raise ValueError('Matrix is not positive')
        else:
            _lib.check(rc)
        self.residuals = list(res[:k + 1])
        self.alphas = list(al[:k])
        self.betas = list(be[:k])
        return xt

    def _solve_host(self, b):
        A, B = self.A, self.B
        applyB = (lambda r: B * r) if B is not None else (lambda r: r.copy())
        x = np.zeros_like(b) if self.initial_guess is None else np.array(self.initial_guess, np.float64)
        r = b - A @ x
        z = applyB(r)
        d = z.copy()
        rz = float(np.dot(r, z))
        if rz < 0:
            raise ValueError('Matrix is not positive')
        residuals = [np.sqrt(rz)]
        alphas, betas = [], []
        tol = self.tolerance * residuals[0] if self.relativeconv else self.tolerance
        norms = [float(np.linalg.norm(r))]
        bnorm = float(np.linalg.norm(b)) or 1.0

        def converged():
            if self.stop_type == 1:
                return norms[-1] <= self.tolerance * bnorm
            return residuals[-1] <= tol

        it = 0
        while not converged() and it < self.maxiter:
            z = A @ d
            dz = float(np.dot(d, z))
            if dz == 0:
                self.breakdown = True
                break
            alpha = rz / dz
            x = x + alpha * d
            r = r - alpha * z
            z = applyB(r)
            rz_prev = rz
            rz = float(np.dot(r, z))
            if rz < 0:
                self.breakdown = True
                warnings.warn('ConjGrad breakdown')
                x = x - alpha * d
                break
            beta = rz / rz_prev
            d = z + beta * d
            residuals.append(np.sqrt(rz))
            norms.append(float(np.linalg.norm(r)))
            alphas.append(alpha)
            betas.append(beta)
            if self.callback is not None:
                self.callback(k=it, x=x, r=r)
            it += 1
        self.residuals, self.alphas, self.betas = residuals, alphas, betas
        self.residual_norms = norms
        return x

    def eigenvalue_estimates(self):
        return lanczos_eigenvalues(self.alphas, self.betas)


class DistConjGrad:
    """ConjGrad on N row-partitioned ranks: the cbc.block loop of
    ``ConjGrad._solve_host`` with every vector a list of local slices, the
    operator and preconditioner applied rank-locally (halo exchanges inside
    them) and each dot product reduced over ranks -- one 8-byte all-reduce
    per dot (RCCL under torch.distributed "nccl" on GPUs, gloo on CPUs).

    spmv(xs, ys) / precond(rs, zs): fill the output slices in place.
    allreduce(float) -> float: sum over ranks (None: no other ranks -- a
    single rank, or all virtual ranks' slices held in this process).
    Local dots are summed in slice order, so a solve is deterministic.
    x0 = 0 (the reference's default); stop_type None: sqrt(<r, B r>) against
    the (absolute unless relativeconv) tolerance; 1: ||r|| <= tol ||b||.
    """

    def __init__(self, spmv, precond, allreduce=None, tolerance=1e-5, maxiter=200, relativeconv=False,
                 stop_type=None):
        self.spmv, self.precond, self.allreduce = spmv, precond, allreduce
        self.tolerance, self.maxiter = tolerance, maxiter
        self.relativeconv, self.stop_type = relativeconv, stop_type
        self.residuals, self.alphas, self.betas, self.residual_norms = [], [], [], []
        self.breakdown = False

    @classmethod
    def for_handles(cls, handles, stream=None, group=None, **kw):
        """PCG for DistMetricAMG handles: one handle per process (RCCL ranks;
        dots all-reduced over ``group`` of the initialised torch.distributed
        world) or a list of virtual rank handles of one process."""
        from .amg import DistMetricAMG
        hs = list(handles) if isinstance(handles, (list, tuple)) else [handles]
        if len(hs) > 1:        # virtual ranks: lockstep, exchanges as device copies
            return cls(lambda xs, ys: DistMetricAMG.virtual_spmv(hs, xs, ys, stream),
                       lambda rs, zs: DistMetricAMG.virtual_apply(hs, rs, zs, stream), None, **kw)
        if hs[0].nranks == 1:
            return cls(lambda xs, ys: hs[0].spmv_device(xs[0], ys[0], stream),
                       lambda rs, zs: hs[0].apply_device(rs[0], zs[0], stream), None, **kw)
        import torch
        import torch.distributed as dist
        h = hs[0]

        dev = 'cpu' if dist.get_backend(group) == 'gloo' else 'cuda'   # gloo: host-staged ranks

        def allreduce(v):
            t = torch.tensor([v], dtype=torch.float64, device=dev)
            dist.all_reduce(t, group=group)
            return float(t.item())
        return cls(lambda xs, ys: h.spmv_device(xs[0], ys[0], stream),
                   lambda rs, zs: h.apply_device(rs[0], zs[0], stream), allreduce, **kw)

    def _dot(self, a, b):
        v = 0.0
        for x, y in zip(a, b):
            v += float((x * y).sum())
        return self.allreduce(v) if self.allreduce is not None else v

    def solve(self, bs):
        """bs: list of local right-hand-side slices (torch tensors); returns
        the list of local solution slices."""
        xs = [b.new_zeros(b.shape) for b in bs]
        rs = [b.clone() for b in bs]
        zs = [b.new_zeros(b.shape) for b in bs]
        qs = [b.new_zeros(b.shape) for b in bs]
        self.precond(rs, zs)
        ds = [z.clone() for z in zs]
        rz = self._dot(rs, zs)
        if rz < 0:
            raise ValueError('Matrix is not positive')
        residuals = [float(np.sqrt(rz))]
        track = self.stop_type == 1          # ||r|| costs one more reduction per iteration
        norms = [float(np.sqrt(self._dot(rs, rs)))] if track else []
        bnorm = (norms[0] if track else 1.0) or 1.0
        alphas, betas = [], []
        tol = self.tolerance * residuals[0] if self.relativeconv else self.tolerance

        def converged():
            if self.stop_type == 1:
                return norms[-1] <= self.tolerance * bnorm
            return residuals[-1] <= tol

        it = 0
        while not converged() and it < self.maxiter:
            self.spmv(ds, qs)
            dq = self._dot(ds, qs)
            if dq == 0:
                self.breakdown = True
                break
            alpha = rz / dq
            for x, d in zip(xs, ds):
                x.add_(d, alpha=alpha)
            for r, q in zip(rs, qs):
                r.sub_(q, alpha=alpha)
            self.precond(rs, zs)
            rz_prev = rz
            rz = self._dot(rs, zs)
            if rz < 0:
                self.breakdown = True
                warnings.warn('ConjGrad breakdown')
                for x, d in zip(xs, ds):
                    x.sub_(d, alpha=alpha)
                break
            beta = rz / rz_prev
            for d, z in zip(ds, zs):
                d.mul_(beta).add_(z)
            residuals.append(float(np.sqrt(rz)))
            if track:
                norms.append(float(np.sqrt(self._dot(rs, rs))))
            alphas.append(alpha)
            betas.append(beta)
            it += 1
        self.residuals, self.alphas, self.betas, self.residual_norms = residuals, alphas, betas, norms
        return xs

    def eigenvalue_estimates(self):
        return lanczos_eigenvalues(self.alphas, self.betas)
