"""Preconditioner factories of the reference's drivers, block form included.

Reference: /root/reference/src/utils.py
  get_block_diag_precond(A, W, bcs)                          :9-12   exact block LU
  get_hazmath_amg_precond(A, W, bcs, parameters, ...)         :15-42  plain (non-metric) AMG
  get_hazmath_metric_precond(A, W, bcs, parameters, idofs)    :45-53  R^T Minv R on a block system
  get_hazmath_metric_precond_mono(A, W, bcs, parameters, idofs) :56-90 metricAMG on the monolithic CSR
  solve_haznics(A, b, W, interface_dofs)                    :95-132 the whole solve in the library
``ii_convert`` (fenics_ii) becomes ``to_monolithic``; ``ReductionOperator``
maps a block vector [x0, x1] onto the monolithic vector (concatenation) and
its transpose splits it back, so ``R.T * Minv * R`` applies the monolithic
preconditioner to block vectors exactly as the reference composes it (:53).
"""
from __future__ import annotations

import numpy as np

from .amg import MetricAMG
from . import parameters as P


def to_monolithic(A):
    """2x2 list of scipy blocks | BlockSystem | sparse -> monolithic CSR (sorted)."""
    import scipy.sparse as sp
    if hasattr(A, 'blocks'):
        A = A.blocks
    elif hasattr(A, 'scipy'):
        A = A.scipy()
    if isinstance(A, (list, tuple)):
        M = sp.bmat(A, format='csr')
    else:
        M = sp.csr_matrix(A)
    M.sort_indices()
    return M


def _sizes(W):
    return [int(w.dim()) if hasattr(w, 'dim') else int(w) for w in W]


class ReductionOperator:
    """Block vector <-> monolithic vector (xii.ReductionOperator([len(W)], W))."""
    _mamg_operator = True      # composes with MetricAMG.__mul__ into a product

    def __init__(self, W, transpose=False):
        self.sizes = _sizes(W)
        self.offsets = np.concatenate([[0], np.cumsum(self.sizes)])
        self.transposed = transpose

    @property
    def T(self):
        return ReductionOperator(self.sizes, not self.transposed)

    def __call__(self, x):
        if self.transposed:                      # monolithic -> blocks
            x = np.asarray(x)
            return [x[self.offsets[i]:self.offsets[i + 1]].copy() for i in range(len(self.sizes))]
        return np.concatenate([np.asarray(xi, dtype=np.float64) for xi in x])

    def __mul__(self, other):
        if isinstance(other, (ReductionOperator, MetricAMG, _Product)):
            return _Product([self, other])
        return self(other)


class _Product:
    """Operator product applied right to left (R.T * Minv * R)."""
    _mamg_operator = True

    def __init__(self, ops):
        self.ops = []
        for o in ops:
            self.ops.extend(o.ops if isinstance(o, _Product) else [o])

    def __mul__(self, other):
        if isinstance(other, (ReductionOperator, MetricAMG, _Product)):
            return _Product([self, other])
        x = other
        for o in reversed(self.ops):
            x = o(x) if isinstance(o, ReductionOperator) else o * x
        return x

    __call__ = __mul__

    @property
    def monolithic(self):
        """the monolithic preconditioner inside (for device-resident PCG)."""
        for o in self.ops:
            if isinstance(o, MetricAMG):
                return o
        return None


def get_hazmath_metric_precond_mono(A, W, bcs=None, parameters=None, interface_dofs=None, **kw):
    """metricAMG(A, W, idofs=interface_dofs, parameters=parameters)  (src/utils.py:56-90).
    ``parameters`` None -> the reference's default dict (src/utils.py:60-82,
    ``parameters.parameters_metric_default``: UA + HEM + W + SGS + scaling +
    SCHWARZ_SYMMETRIC on the seeds' 2-rings, which runs as SCHWARZ_RINGS).  A
    dict is used as given (parameters_metric_schwarz: node patches on level 0;
    ``parameters_metric_mi355x``: the GPU profile, an explicit opt-in); a
    component this build lacks (MWM/HEC aggregation, AMLI) raises MamgError;
    ``parameters.to_gpu_profile`` is the explicit opt-in mapping."""
    if parameters is None:
        parameters = P.parameters_metric_default
    B = MetricAMG(A, W, idofs=interface_dofs, parameters=parameters, **kw)
    B.substitutions = []
    return B


def get_hazmath_metric_precond(A, W, bcs=None, parameters=None, interface_dofs=None, **kw):
    """R^T * Minv * R with Minv the monolithic metric AMG (src/utils.py:45-53)."""
    AA = to_monolithic(A)
    R = ReductionOperator(W)
    Minv = get_hazmath_metric_precond_mono(AA, W, bcs, parameters=parameters,
                                           interface_dofs=interface_dofs, **kw)
    op = R.T * Minv * R
    op.Aop = AA
    return op


def get_hazmath_amg_precond(A, W=None, bcs=None, parameters=None, interface_dofs=None, **kw):
    """Plain (non-metric) AMG on the monolithic matrix (src/utils.py:15-42):
    no interface seeds.  ``parameters`` None -> the reference's default dict
    (src/utils.py:20-38, ``parameters.parameters_amg_default``: UA + VMB + W +
    SGS + scaling).

    Substitution: the reference's AMGhaz (src/utils.py:40) never
    receives W, so HAZmath aggregates point-wise there.  Here W, when given,
    makes the hierarchy nodal (num_functions = the number of equal blocks:
    nodal aggregation and node-block SGS, the only SGS this build has);
    ``num_functions=1`` gives point-wise aggregation with a point smoother
    (SGS then needs a Jacobi-family ``smoother``: this build's SGS is the
    node-block multicolour one, so a point-wise default would substitute the
    smoother instead).  The choice is recorded in ``.substitutions`` instead
    of the num_functions warning on every call; every other warning of the
    construction still reaches the caller."""
    import warnings
    params = dict(P.parameters_amg_default) if parameters is None else dict(parameters)
    params['Schwarz_levels'] = 0
    with warnings.catch_warnings():
        warnings.filterwarnings('ignore', message=r'num_functions -> ', category=UserWarning)
        B = MetricAMG(to_monolithic(A), W, idofs=None, parameters=params, **kw)
    B.substitutions = [n for n in getattr(B, 'notes', [])] + (
        ['nodal hierarchy from W (the reference AMGhaz gets no W: point-wise aggregation there)']
        if B.params.num_functions > 1 and 'num_functions' not in kw and 'num_functions' not in params else [])
    return B


def solve_haznics(A, b, W, interface_dofs=None, parameters=None, tolerance=1e-8, maxiter=500):
    """The whole solve in the library (src/utils.py:95-132: haznics'
    fenics_metric_amg_solver_dcsr on the monolithic matrix): metric AMG seeded
    at interface_dofs + PCG, both on the device.  HAZmath's solver reads its
    own defaults, which are not in the reference tree; here ``parameters``
    (default: the GPU profile) and the drivers' CG tolerance apply.
    Returns (niters, [x0, x1], solve seconds) -- x split by W like the
    reference's ii_Function."""
    import time
    from .krylov import ConjGrad
    AA = to_monolithic(A)
    sizes = _sizes(W)
    t0 = time.time()
    B = get_hazmath_metric_precond_mono(AA, sizes, parameters=parameters, interface_dofs=interface_dofs,
                                        num_functions=2 if len(sizes) == 2 and sizes[0] == sizes[1] else 1)
    cg = ConjGrad(AA, precond=B, tolerance=tolerance, maxiter=maxiter)   # same A: device PCG
    bb = np.concatenate([np.asarray(v, np.float64) for v in b]) if isinstance(b, (list, tuple)) \
        else np.asarray(b, np.float64)
    x = cg * bb
    x = x.cpu().numpy() if hasattr(x, 'cpu') else np.asarray(x)
    dt = time.time() - t0
    offs = np.cumsum([0] + list(sizes))
    return len(cg.residuals) - 1, [x[offs[i]:offs[i + 1]] for i in range(len(sizes))], dt


class BlockDiagLU:
    """Exact LU of each diagonal block (src/utils.py:9-12, PETSc LU there;
    SuperLU here).  The 'diag' option of the EMI / bidomain drivers -- a
    reference baseline, not part of the metric-AMG hot path."""

    def __init__(self, A, W):
        from scipy.sparse.linalg import splu
        AA = to_monolithic(A)
        self.sizes = _sizes(W)
        off = np.concatenate([[0], np.cumsum(self.sizes)])
        self.off = off
        self.lu = [splu(AA[off[i]:off[i + 1], off[i]:off[i + 1]].tocsc()) for i in range(len(self.sizes))]

    def __mul__(self, r):
        if isinstance(r, (list, tuple)):
            return [lu.solve(np.asarray(ri)) for lu, ri in zip(self.lu, r)]
        r = np.asarray(r)
        return np.concatenate([lu.solve(r[self.off[i]:self.off[i + 1]]) for i, lu in enumerate(self.lu)])

    __call__ = __mul__


def get_block_diag_precond(A, W, bcs=None):
    return BlockDiagLU(A, W)
