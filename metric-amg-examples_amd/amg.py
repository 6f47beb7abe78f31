"""MetricAMG: drop-in for cbc.block's ``block.algebraic.hazmath.metricAMG``.

Reference call sites:
  Minv = metricAMG(A, W, idofs=interface_dofs, parameters=parameters)
      /root/reference/src/utils.py:86   (without idofs :88)
  R.T * Minv * R                        src/utils.py:53 (block form)
  ConjGrad(AA_, precond=BB, ...)        src/bidomain_3d.py:149
``MetricAMG`` runs the host setup + upload through libmamg's C-ABI
(``mamg_setup``) and applies one multigrid cycle per ``B * r`` on the GPU
(``mamg_apply`` / ``mamg_apply_device``).  There is no CPU fallback: without
libmamg.so or a HIP device the constructor raises.
"""
from __future__ import annotations

import ctypes as C
import warnings

import numpy as np

from . import _lib
from .parameters import make_params, params_to_dict


def csr_arrays(A):
    """scipy sparse | (indptr, indices, data[, shape]) | problems.System ->
    (indptr int64, indices int32, data float64, nrows, ncols), sorted."""
    if hasattr(A, 'indptr') and hasattr(A, 'indices') and hasattr(A, 'data') \
            and not hasattr(A, 'tocsr'):
        indptr, indices, data = A.indptr, A.indices, A.data
        n = len(indptr) - 1
        shape = (n, n)
    elif hasattr(A, 'tocsr'):
        M = A.tocsr()
        if not M.has_sorted_indices:
            M = M.sorted_indices()
        indptr, indices, data, shape = M.indptr, M.indices, M.data, M.shape
    else:
        indptr, indices, data = A[0], A[1], A[2]
        n = len(indptr) - 1
        shape = A[3] if len(A) > 3 else (n, n)
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    data = np.ascontiguousarray(data, dtype=np.float64)
    if indptr.ndim != 1 or len(indptr) != shape[0] + 1 or indptr[0] != 0 \
            or len(indices) != indptr[-1] or len(data) != indptr[-1]:
        raise ValueError('inconsistent CSR arrays: len(indptr)=%d, indptr[-1]=%d, '
                         'len(indices)=%d, len(data)=%d'
                         % (len(indptr), indptr[-1], len(indices), len(data)))
    return indptr, indices, data, int(shape[0]), int(shape[1])


def _dims(W, n):
    if W is None:
        return [n]
    dims = []
    for w in W:
        dims.append(int(w.dim()) if hasattr(w, 'dim') else int(w))
    if sum(dims) != n:
        raise ValueError('sum of W dims %d != matrix size %d' % (sum(dims), n))
    return dims


def _with_functions(W, parameters, overrides):
    """The reference's metricAMG receives the block space W (src/utils.py:86):
    a W of k >= 2 equal-sized blocks (the bidomain's and EMI's P1 x P1) gives
    num_functions = k unless the dict or an override sets it.

    Returns (overrides, notes).  Whether HAZmath's metricAMG itself derives
    num_functions from W is not pinned by the reference source, so the
    inference is reported: as a note (MetricAMG.notes) and, when the caller
    passed a dict without num_functions (a reference preset such as
    parameters_standard, which would otherwise aggregate point-wise), as a
    UserWarning.  A caller-supplied num_functions (dict or keyword) always
    wins."""
    if 'num_functions' in overrides or (parameters and 'num_functions' in parameters) \
            or W is None or not isinstance(W, (list, tuple)) or len(W) < 2:
        return overrides, []
    dims = [int(w.dim()) if hasattr(w, 'dim') else int(w) for w in W]
    if len(set(dims)) != 1:
        return overrides, []
    note = ('num_functions -> %d (inferred from W: %d equal blocks of %d dofs; '
            'pass num_functions=1 for point-wise aggregation)' % (len(dims), len(dims), dims[0]))
    if parameters:
        warnings.warn(note, UserWarning, stacklevel=3)
    return dict(overrides, num_functions=len(dims)), [note]


def _device_ptr(x):
    """(pointer, keepalive) for a torch CUDA tensor / object with data_ptr()."""
    if hasattr(x, 'data_ptr') and getattr(x, 'is_cuda', False):
        if x.dtype.__str__() != 'torch.float64' or not x.is_contiguous():
            raise TypeError('device vectors must be contiguous float64')
        return C.c_void_p(x.data_ptr())
    if isinstance(x, int):
        return C.c_void_p(x)
    raise TypeError('expected a CUDA tensor or a raw device pointer')


def _stream_ptr(stream):
    if stream is None:
        return None
    if hasattr(stream, 'cuda_stream'):
        return C.c_void_p(stream.cuda_stream)
    return C.c_void_p(int(stream))


def gpu_setup_supported(p) -> bool:
    """The GPU setup (mamg_setup_gpu) covers num_functions 1 and 2: node-block,
    general seed-block, overlapping-ring (SCHWARZ_ADDITIVE) and point smoothers,
    nodal or point SA (csrc/gsetup.hip).  What it still refuses at run time
    (MAMG_ERR_UNSUPPORTED) 'auto' hands to the host setup."""
    return p.num_functions in (1, 2)


def _device_csr(A):
    """(indptr, indices, data[, shape]) of CUDA tensors -> (mamg_csr, n, m) or None."""
    if not isinstance(A, (tuple, list)) or len(A) < 3 or not getattr(A[0], 'is_cuda', False):
        return None
    ip, ix, dv = A[0], A[1], A[2]
    import torch
    if ip.dtype != torch.int64 or ix.dtype != torch.int32 or dv.dtype != torch.float64 \
            or not (ip.is_contiguous() and ix.is_contiguous() and dv.is_contiguous()):
        raise TypeError('device CSR must be contiguous int64 indptr, int32 indices, float64 data')
    n = ip.numel() - 1
    shape = A[3] if len(A) > 3 else (n, n)
    s = _lib.mamg_csr()
    s.nrows, s.ncols, s.nnz = n, int(shape[1]), ix.numel()
    s.rowptr = C.cast(C.c_void_p(ip.data_ptr()), C.POINTER(C.c_int64))
    s.colind = C.cast(C.c_void_p(ix.data_ptr()), C.POINTER(C.c_int32))
    s.values = C.cast(C.c_void_p(dv.data_ptr()), C.POINTER(C.c_double))
    return s, n, int(shape[1])


class MetricAMG:
    """One multigrid cycle per application, on the GPU.

    A: CSR operator (scipy sparse, (indptr, indices, data), or System), or a
       tuple of CUDA tensors (indptr int64, indices int32, data float64) that
       is already in HBM (GPU setup only; read during setup, not kept).
    W: list of function spaces / block sizes (only sizes are used).
    idofs: interface dofs seeding the level-0 Schwarz blocks (src/utils.py:84).
    parameters: dict with the reference's key names (see parameters.py).
    setup: 'gpu' (mamg_setup_gpu: hierarchy built by gfx950 kernels, bitwise
       equal to the host setup), 'host' (mamg_setup: C++/OpenMP setup, then
       upload), or 'auto' (default): 'gpu' when the profile is one the GPU
       setup covers, else 'host'.  ``setup_path`` records what ran and why.
    """

    def __init__(self, A, W=None, idofs=None, parameters=None, setup='auto', **overrides):
        self._L = _lib.lib()
        ov, self.notes = _with_functions(W, parameters, overrides)
        self.params = make_params(parameters, **ov)
        if idofs is not None:
            self.idofs = np.ascontiguousarray(idofs, dtype=np.int32)
            ip, ni = _lib.ptr(self.idofs, C.c_int32), len(self.idofs)
        else:
            self.idofs, ip, ni = None, None, 0
        if setup not in ('auto', 'gpu', 'host'):
            raise ValueError("setup must be 'auto', 'gpu' or 'host'")
        h = C.c_void_p()
        dev = _device_csr(A)
        if dev is not None:                      # A already in HBM
            csr, n, m = dev
            if n != m:
                raise ValueError('A must be square')
            if setup == 'host':
                raise ValueError("a device-resident A needs setup='gpu' (or 'auto')")
            self.shape = (n, n)
            self.W = _dims(W, n)
            self._A = None
            self._Aop = None
            _lib.check(self._L.mamg_setup_gpu_device(C.byref(csr), ip, ni, C.byref(self.params),
                                                     C.byref(h)))
            self._h = h
            self.setup_path = 'gpu'
            return
        indptr, indices, data, n, m = csr_arrays(A)
        if n != m:
            raise ValueError('A must be square')
        self.shape = (n, n)
        self.W = _dims(W, n)
        self._A = (indptr, indices, data)        # level 0 stays referenced
        self._Aop = A
        csr = _lib.as_csr_struct(indptr, indices, data, m)
        use_gpu = setup == 'gpu' or (setup == 'auto' and gpu_setup_supported(self.params))
        self.setup_path = 'host'
        if use_gpu:
            rc = self._L.mamg_setup_gpu(C.byref(csr), ip, ni, C.byref(self.params), C.byref(h))
            if rc == _lib.ERR_UNSUPPORTED and setup == 'auto':
                # e.g. seed blocks that are not node-aligned: the host setup
                # builds the same profile; recorded, not silent
                self.setup_path = 'host (%s)' % self._L.mamg_last_error().decode(errors='replace')
            else:
                _lib.check(rc)
                self.setup_path = 'gpu'
        if not self.setup_path == 'gpu':
            _lib.check(self._L.mamg_setup(C.byref(csr), ip, ni, C.byref(self.params), C.byref(h)))
        self._h = h

    @property
    def setup_timings(self) -> dict:
        """GPU setup phase timings in ms (zeros for a host setup)."""
        ms = (C.c_double * 8)()
        _lib.check(self._L.mamg_setup_timings(self._h, ms))
        names = ('aggregate', 'smoother', 'prolongator', 'galerkin', 'coarsest', 'layout',
                 'setup_total', 'upload_A0')
        out = {k: round(ms[i], 3) for i, k in enumerate(names)}
        lm = (C.c_double * 4)()
        _lib.check(self._L.mamg_layout_timings(self._h, lm))
        for i, k in enumerate(('layout_build', 'layout_kregion', 'layout_rehome', 'layout_finish')):
            out[k] = round(lm[i], 3)
        return out

    @classmethod
    def from_host(cls, H: 'HostHierarchy', W=None):
        """Upload an existing HostHierarchy (``mamg_upload``) instead of
        running the setup again."""
        self = cls.__new__(cls)
        self._L = _lib.lib()
        indptr, indices, data = H._A
        n = len(indptr) - 1
        self.shape = (n, n)
        self.W = _dims(W, n)
        self.params = H.params
        self._A = H._A
        self._Aop = None
        self.idofs = H.idofs
        csr = _lib.as_csr_struct(indptr, indices, data, n)
        h = C.c_void_p()
        _lib.check(self._L.mamg_upload(H._h, C.byref(csr), C.byref(self.params), C.byref(h)))
        self._h = h
        return self

    # -- properties --------------------------------------------------------
    @property
    def handle(self):
        return self._h

    @property
    def num_levels(self) -> int:
        return self._L.mamg_num_levels(self._h)

    @property
    def layout(self) -> str:
        """device layout: 'csr' (general) or 'bsr2' (nodal, 2 fields)."""
        return ('csr', 'bsr2')[self._L.mamg_device_layout(self._h)]

    def level_format(self, level: int) -> dict:
        """Device storage of level ``level`` (BSR2 layout): sliced-ELL rows,
        symmetric 2x2 blocks, fused [P | AP] post-smoothing."""
        f = self._L.mamg_level_format(self._h, int(level))
        _lib.check(min(f, 0))
        return {'sell': bool(f & 1), 'sym': bool(f & 2), 'post_fused': bool(f & 4),
                'post_k': bool(f & 8), 'post_sell': bool(f & 16), 'half': bool(f & 32),
                'bands': bool(f & 64), 'patches': bool(f & 128), 'gs': bool(f & 256),
                'rings': bool(f & 512), 'r_bands': bool(f & 1024), 'k_col16': bool(f & 2048)}

    @property
    def kregion(self) -> dict:
        """Placement of the level-0 K values chosen at upload: K ms per
        candidate memory region and the index kept (mamg_kregion_info)."""
        ms = (C.c_double * 16)()
        n, kept = C.c_int(), C.c_int()
        _lib.check(self._L.mamg_kregion_info(self._h, ms, 16, C.byref(n), C.byref(kept)))
        return {'candidates_ms': [round(ms[i], 4) for i in range(min(n.value, 16))], 'kept': kept.value}

    @property
    def effective_params(self) -> dict:
        """The parameters the handle runs, after the reference's Schwarz
        names are resolved (mamg_handle_params)."""
        p = _lib.mamg_params()
        _lib.check(self._L.mamg_handle_params(self._h, C.byref(p)))
        return params_to_dict(p)

    @property
    def apply_bytes(self) -> float:
        b = C.c_double()
        _lib.check(self._L.mamg_apply_bytes(self._h, C.byref(b)))
        return b.value

    # -- application -------------------------------------------------------
    def matvec(self, r):
        """z = B r.  numpy in -> numpy out (host copies); CUDA tensor in ->
        CUDA tensor out (device-resident, current torch stream)."""
        if isinstance(r, np.ndarray):
            rr = np.ascontiguousarray(r, dtype=np.float64)
            if rr.shape != (self.shape[0],):
                raise ValueError('vector size mismatch')
            z = np.empty_like(rr)
            _lib.check(self._L.mamg_apply(self._h, _lib.ptr(rr, C.c_double),
                                          _lib.ptr(z, C.c_double)))
            return z
        import torch
        z = torch.empty_like(r)
        self.apply_device(r, z, torch.cuda.current_stream())
        return z

    def apply_device(self, r, z, stream=None):
        _lib.check(self._L.mamg_apply_device(self._h, _device_ptr(r), _device_ptr(z),
                                             _stream_ptr(stream)))
        return z

    def spmv_device(self, x, y, stream=None):
        _lib.check(self._L.mamg_spmv_device(self._h, _device_ptr(x), _device_ptr(y),
                                            _stream_ptr(stream)))
        return y

    def __mul__(self, r):
        if getattr(r, '_mamg_operator', False):      # Minv * R (block form, src/utils.py:53)
            from .precond import _Product
            return _Product([self, r])
        return self.matvec(r)

    __call__ = matvec

    def time_apply(self, r, z, reps, mode=0, stream=None):
        """(ms per apply, kernel_ms[16], class_bytes[16]) via HIP events."""
        ms = C.c_double()
        kms = (C.c_double * 16)()
        cb = (C.c_double * 16)()
        _lib.check(self._L.mamg_time_apply(self._h, _device_ptr(r), _device_ptr(z), int(reps),
                                           int(mode), C.byref(ms), kms, cb, _stream_ptr(stream)))
        return ms.value, list(kms), list(cb)

    def close(self):
        if getattr(self, '_h', None):
            self._L.mamg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


metricAMG = MetricAMG     # the reference's spelling (src/utils.py:2,86)


class HostHierarchy:
    """Host-only setup (``mamg_host_setup``): the hierarchy the device path
    uploads, exported level by level.  Used by tests and the bench's CPU
    baseline; needs no GPU."""

    def __init__(self, A, idofs=None, parameters=None, gpu=False, **overrides):
        self._L = _lib.lib()
        indptr, indices, data, n, m = csr_arrays(A)
        self._A = (indptr, indices, data)
        self.params = make_params(parameters, **overrides)
        csr = _lib.as_csr_struct(indptr, indices, data, m)
        self._csr = csr
        if idofs is not None:
            self.idofs = np.ascontiguousarray(idofs, dtype=np.int32)
            ip, ni = _lib.ptr(self.idofs, C.c_int32), len(self.idofs)
        else:
            self.idofs, ip, ni = None, None, 0
        h = C.c_void_p()
        # gpu=True: the same hierarchy built by the GPU setup, copied back
        # (mamg_gpu_host_setup; bitwise-parity tests and multi-GPU planning)
        fn = self._L.mamg_gpu_host_setup if gpu else self._L.mamg_host_setup
        _lib.check(fn(C.byref(csr), ip, ni, C.byref(self.params), C.byref(h)))
        self._h = h

    @property
    def effective_params(self) -> dict:
        """The parameters the setup ran with (mamg_hier_params)."""
        p = _lib.mamg_params()
        _lib.check(self._L.mamg_hier_params(self._h, C.byref(p)))
        return params_to_dict(p)

    @property
    def num_levels(self):
        return self._L.mamg_hier_num_levels(self._h)

    def sizes(self, l):
        s = (C.c_int64 * 6)()
        _lib.check(self._L.mamg_hier_level_sizes(self._h, l, s))
        return dict(n=s[0], nnzA=s[1], nnzP=s[2], nnzR=s[3], nnzW=s[4], ncoarse=s[5])

    def level(self, l, with_A=True):
        """dict of numpy arrays for level l (A, P, R, WB as (indptr, indices,
        data, shape); winv; agg; Ainv)."""
        s = self.sizes(l)
        n, nc = s['n'], s['ncoarse']
        out = {}

        def alloc(nr, nnz):
            return (np.zeros(nr + 1, np.int64), np.zeros(nnz, np.int32), np.zeros(nnz, np.float64))

        A = alloc(n, s['nnzA']) if with_A else (None, None, None)
        coarsest = nc == 0
        P = alloc(n, s['nnzP']) if not coarsest else (None, None, None)
        R = alloc(nc, s['nnzR']) if not coarsest else (None, None, None)
        Wb = alloc(n, s['nnzW']) if s['nnzW'] else (None, None, None)
        winv = np.zeros(n) if (not coarsest and not s['nnzW']) else None
        agg = np.zeros(n // max(1, self.params.num_functions), np.int64) if not coarsest else None
        Ainv = np.zeros(n * n) if coarsest else None

        def p(a, t):
            return None if a is None else _lib.ptr(a, t)

        args = []
        for M in (A, P, R, Wb):
            args += [p(M[0], C.c_int64), p(M[1], C.c_int32), p(M[2], C.c_double)]
        _lib.check(self._L.mamg_hier_level_export(
            self._h, l, *args, p(winv, C.c_double), p(agg, C.c_int64), p(Ainv, C.c_double)))
        if with_A:
            out['A'] = A + ((n, n),)
        if not coarsest:
            out['P'] = P + ((n, nc),)
            out['R'] = R + ((nc, n),)
            out['agg'] = agg
        if s['nnzW']:
            out['WB'] = Wb + ((n, n),)
        if winv is not None:
            out['winv'] = winv
        if Ainv is not None:
            out['Ainv'] = Ainv.reshape(n, n)
        out['n'] = n
        return out

    def close(self):
        if getattr(self, '_h', None):
            self._L.mamg_hier_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DistPlan:
    """Rank-local partition plan of the multi-GPU V-cycle (``mamg_hier_dist_plan``):
    node ranges, ghost / send lists and rank-local 2x2-block matrices per level."""

    def __init__(self, H: HostHierarchy, rank: int, nranks: int, rep_nodes: int = 32768):
        self._L = _lib.lib()
        self.H = H
        self.rank, self.nranks = rank, nranks
        h = C.c_void_p()
        _lib.check(self._L.mamg_hier_dist_plan(H._h, rank, nranks, rep_nodes, C.byref(h)))
        self._h = h

    @property
    def num_levels(self):
        return self._L.mamg_plan_num_levels(self._h)

    def level(self, l):
        s = (C.c_int64 * 16)()
        _lib.check(self._L.mamg_plan_level_sizes(self._h, l, s))
        (nv, rep, coarsest, o0, o1, ng, ns, nbA, nrA, ncA, nbP, nrP, ncP, nbR, nrR, ncR) = list(s)
        nr = self.nranks
        out = dict(nv=nv, replicated=bool(rep), coarsest=bool(coarsest), o0=o0, o1=o1,
                   nloc=o1 - o0, ghosts=np.zeros(ng, np.int64), ghost_off=np.zeros(nr + 1, np.int64),
                   send_idx=np.zeros(ns, np.int64), send_off=np.zeros(nr + 1, np.int64))

        def alloc(nb, nrows):
            return (np.zeros(nrows + 1, np.int64), np.zeros(nb, np.int32), np.zeros(4 * nb))

        A = alloc(nbA, nrA)
        P = alloc(nbP, nrP) if nrP else (None, None, None)
        R = alloc(nbR, nrR) if nrR else (None, None, None)
        W = np.zeros(4 * (o1 - o0)) if not coarsest else None

        def p(a, t):
            return None if a is None else _lib.ptr(a, t)

        args = []
        for M in (A, P, R):
            args += [p(M[0], C.c_int64), p(M[1], C.c_int32), p(M[2], C.c_double)]
        _lib.check(self._L.mamg_plan_level_export(
            self._h, l, p(out['ghosts'], C.c_int64), p(out['ghost_off'], C.c_int64),
            p(out['send_idx'], C.c_int64), p(out['send_off'], C.c_int64), *args,
            p(W, C.c_double)))
        out['A'] = (A[0], A[1], A[2].reshape(-1, 2, 2), nrA, ncA)
        if nrP:
            out['P'] = (P[0], P[1], P[2].reshape(-1, 2, 2), nrP, ncP)
            out['R'] = (R[0], R[1], R[2].reshape(-1, 2, 2), nrR, ncR)
        if W is not None:
            out['W'] = W.reshape(-1, 2, 2)
        return out

    def close(self):
        if getattr(self, '_h', None):
            self._L.mamg_plan_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GlooExchange:
    """mamg_exchange over the initialised torch.distributed group (gloo, CPU
    tensors): point-to-point isend/irecv per peer, all-reduce as an
    all-gather summed in rank order (deterministic, like the reverse-add)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.d, self.group = dist, group

    def sendrecv(self, sends, counts):
        import torch
        reqs, bufs = [], {}
        for q, n in counts.items():
            bufs[q] = torch.empty(int(n), dtype=torch.float64)
            reqs.append(self.d.irecv(bufs[q], src=q, group=self.group))
        for q, a in sends.items():
            reqs.append(self.d.isend(torch.from_numpy(np.ascontiguousarray(a)), dst=q, group=self.group))
        for r in reqs:
            r.wait()
        return {q: b.numpy() for q, b in bufs.items()}

    def allreduce(self, a):
        import torch
        n = self.d.get_world_size(self.group)
        parts = [torch.empty(a.size, dtype=torch.float64) for _ in range(n)]
        self.d.all_gather(parts, torch.from_numpy(np.ascontiguousarray(a)), group=self.group)
        out = parts[0].numpy().copy()
        for p in parts[1:]:
            out += p.numpy()
        return out


class DistMetricAMG:
    """Multi-GPU preconditioner: one process per GPU (``mamg_setup_dist``).

    Every rank passes the same global A (the deterministic setup is
    replicated) -- a host CSR, or a tuple of CUDA tensors already in HBM
    (``problems.bidomain_device``: no rank then holds the global matrix on the
    host, ``mamg_setup_dist_device``) -- and applies B to its local slice r_local = [u1(o0:o1);
    u2(o0:o1)] (field-major, length 2*(o1-o0)).  comm_id: bytes from
    ``DistMetricAMG.unique_id()`` on rank 0, broadcast to all ranks; None
    builds a virtual (single-GPU, no RCCL) rank for tests."""

    def __init__(self, A, W=None, idofs=None, parameters=None, rank=0, nranks=1, comm_id=None,
                 rep_nodes=32768, exchange=None, **overrides):
        self._L = _lib.lib()
        dev = _device_csr(A)
        if dev is not None:                      # A_0 already in HBM (mamg_setup_dist_device)
            csr, n, m = dev
            self._A = None
        else:
            indptr, indices, data, n, m = csr_arrays(A)
            self._A = (indptr, indices, data)
            csr = _lib.as_csr_struct(indptr, indices, data, m)
        self.shape = (n, n)
        self.W = _dims(W, n)
        ov, self.notes = _with_functions(W, parameters, overrides)
        self.params = make_params(parameters, **ov)
        if idofs is not None:
            self.idofs = np.ascontiguousarray(idofs, dtype=np.int32)
            ip, ni = _lib.ptr(self.idofs, C.c_int32), len(self.idofs)
        else:
            self.idofs, ip, ni = None, None, 0
        h = C.c_void_p()
        setup = self._L.mamg_setup_dist_device if dev is not None else self._L.mamg_setup_dist
        _lib.check(setup(C.byref(csr), ip, ni, C.byref(self.params), rank, nranks,
                         comm_id, int(rep_nodes), C.byref(h)))
        self._h = h
        self.rank, self.nranks = rank, nranks
        self._exchange = None
        if exchange is not None:
            if comm_id is not None:
                raise ValueError('exchange= replaces the RCCL communicator: pass comm_id=None')
            self.set_exchange(exchange)
        o0, o1, nv = C.c_int64(), C.c_int64(), C.c_int64()
        _lib.check(self._L.mamg_dist_range(h, C.byref(o0), C.byref(o1), C.byref(nv)))
        self.o0, self.o1, self.nv = o0.value, o1.value, nv.value

    def set_exchange(self, exchange):
        """Host-staged transport (mamg_dist_set_exchange): 'gloo' = the
        initialised torch.distributed process group (CPU tensors), or an
        object with sendrecv(sends, recv_counts) -> {q: ndarray} and
        allreduce(ndarray) -> ndarray.  The device kernels and the exchange
        schedule are the RCCL path's."""
        ex = GlooExchange() if exchange == 'gloo' else exchange
        me, P = self.rank, self.nranks

        def sendrecv(ctx, n, send, scount, recv, rcount):
            try:
                sends = {q: np.ctypeslib.as_array(send[q], (scount[q],)) for q in range(n)
                         if q != me and scount[q] > 0}
                counts = {q: rcount[q] for q in range(n) if q != me and rcount[q] > 0}
                got = ex.sendrecv(sends, counts)
                for q, a in got.items():
                    np.ctypeslib.as_array(recv[q], (counts[q],))[:] = a
                return 0
            except Exception:          # noqa: BLE001 -- reported through the status code
                import traceback
                traceback.print_exc()
                return 1

        def allreduce(ctx, buf, count):
            try:
                a = np.ctypeslib.as_array(buf, (count,))
                a[:] = ex.allreduce(a.copy())
                return 0
            except Exception:          # noqa: BLE001
                import traceback
                traceback.print_exc()
                return 1
        fns = (_lib.SENDRECV_FN(sendrecv), _lib.ALLREDUCE_FN(allreduce))
        st = _lib.mamg_exchange(None, fns[0], fns[1])
        _lib.check(self._L.mamg_dist_set_exchange(self._h, C.byref(st)))
        self._exchange = (ex, fns, st)          # the callbacks must outlive the handle's use
        assert P == self.nranks

    @staticmethod
    def unique_id() -> bytes:
        L = _lib.lib()
        buf = C.create_string_buffer(L.mamg_comm_id_bytes())
        _lib.check(L.mamg_comm_unique_id(buf))
        return buf.raw

    @property
    def nloc(self):
        return self.o1 - self.o0

    def local_slice(self, v):
        return np.concatenate([v[self.o0:self.o1], v[self.nv + self.o0:self.nv + self.o1]])

    @property
    def apply_bytes(self):
        b = C.c_double()
        _lib.check(self._L.mamg_dist_apply_bytes(self._h, C.byref(b)))
        return b.value

    @property
    def apply_launches(self):
        """{'kernels', 'p2p_groups', 'p2p_messages', 'allreduces', 'stream_forks'}
        one apply issues on this rank (mamg_dist_apply_launches)."""
        c = (C.c_int64 * 5)()
        _lib.check(self._L.mamg_dist_apply_launches(self._h, c))
        return dict(zip(('kernels', 'p2p_groups', 'p2p_messages', 'allreduces', 'stream_forks'), list(c)))

    def apply_device(self, r, z, stream=None):
        _lib.check(self._L.mamg_dist_apply_device(self._h, _device_ptr(r), _device_ptr(z),
                                                  _stream_ptr(stream)))
        return z

    def apply_graph(self, r, z, stream=None):
        """The apply replayed from a hipGraph (mamg_dist_apply_graph: captured
        on first use per (r, z), RCCL calls inside the capture).  Raises
        MamgError (MAMG_ERR_UNSUPPORTED) for host-staged / virtual exchanges
        or after a failed capture; apply_device stays the eager path."""
        _lib.check(self._L.mamg_dist_apply_graph(self._h, _device_ptr(r), _device_ptr(z), _stream_ptr(stream)))
        return z

    def prepare_graph(self, r, z):
        """Capture (or find) the apply's hipGraph for (r, z) without launching
        it (mamg_dist_graph_prepare).  Returns None on success, else the
        library's message (the handle then stays eager)."""
        rc = self._L.mamg_dist_graph_prepare(self._h, _device_ptr(r), _device_ptr(z))
        return None if rc == 0 else self._L.mamg_last_error().decode(errors='replace')

    def time_apply(self, r, z, reps, mode=0, stream=None):
        """mode 0: eager, events around the level-0 residual and K; 1: eager,
        events around every op; 2: graph replays (kernel_ms zero)."""
        ms = C.c_double()
        kms = (C.c_double * 16)()
        cb = (C.c_double * 16)()
        _lib.check(self._L.mamg_dist_time_apply(self._h, _device_ptr(r), _device_ptr(z), int(reps),
                                                int(mode), C.byref(ms), kms, cb, _stream_ptr(stream)))
        return ms.value, list(kms), list(cb)

    def spmv_device(self, x, y, stream=None):
        """y = A x on this rank's rows (local field-major slices; one halo
        exchange of x)."""
        _lib.check(self._L.mamg_dist_spmv_device(self._h, _device_ptr(x), _device_ptr(y),
                                                 _stream_ptr(stream)))
        return y

    @staticmethod
    def virtual_spmv(handles, xs, ys, stream=None):
        n = len(handles)
        H = (C.c_void_p * n)(*[h._h.value for h in handles])
        X = (C.c_void_p * n)(*[_device_ptr(x).value for x in xs])
        Y = (C.c_void_p * n)(*[_device_ptr(y).value for y in ys])
        _lib.check(_lib.lib().mamg_dist_virtual_spmv(H, n, X, Y, _stream_ptr(stream)))

    @staticmethod
    def virtual_apply(handles, rs, zs, stream=None, graph=False):
        """graph=True: the lockstep apply captured into one hipGraph and
        replayed (mamg_dist_virtual_apply_graph)."""
        n = len(handles)
        H = (C.c_void_p * n)(*[h._h.value for h in handles])
        R = (C.c_void_p * n)(*[_device_ptr(r).value for r in rs])
        Z = (C.c_void_p * n)(*[_device_ptr(z).value for z in zs])
        f = _lib.lib().mamg_dist_virtual_apply_graph if graph else _lib.lib().mamg_dist_virtual_apply
        _lib.check(f(H, n, R, Z, _stream_ptr(stream)))

    def close(self):
        if getattr(self, '_h', None):
            self._L.mamg_dist_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
