"""Synthetic inputs of the reference's benchmark configurations.

The reference assembles its systems with legacy FEniCS + fenics_ii
(src/bidomain_2d.py:51-99, meshes src/utils.py:149-182); neither exists here,
so libmamg's C++ generator restates the same P1 matrices on dolfin's
structured meshes.  Mesh loops follow the drivers:
2-D n = 2^i, i in [5, 5+nrefs) (src/bidomain_2d.py:168); 3-D i in [3, 3+nrefs)
(src/bidomain_3d.py:113).  The benchmark uses the finest level.
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np

from . import _lib


@dataclasses.dataclass
class System:
    indptr: np.ndarray        # int64 [N+1]
    indices: np.ndarray       # int32 [nnz]
    data: np.ndarray          # float64 [nnz]
    N: int
    nv: int                   # dofs per field (W[0].dim() == W[1].dim())
    dim: int
    n: int
    gamma: float

    @property
    def idofs(self) -> np.ndarray:
        """interface dofs = the u2 block (src/bidomain_3d.py:138)."""
        return np.arange(self.nv, 2 * self.nv, dtype=np.int32)

    @property
    def W(self):
        return [self.nv, self.nv]

    @property
    def nnz(self):
        return int(self.indptr[-1])

    def scipy(self):
        import scipy.sparse as sp
        A = sp.csr_matrix((self.data, self.indices, self.indptr), shape=(self.N, self.N))
        A.has_sorted_indices = True
        return A


def finest_n(dim: int, nrefs: int) -> int:
    return 2 ** ((5 if dim == 2 else 3) + nrefs - 1)


def bidomain(dim: int, n: int, gamma: float, kappa1: float = 2.0, kappa2: float = 3.0) -> System:
    """Monolithic [[k1 K + g M, -g M], [-g M, k2 K + g M]] on UnitSquare/Cube(n)."""
    L = _lib.lib()
    N, nnz = C.c_int64(), C.c_int64()
    _lib.check(L.mamg_gen_bidomain_size(dim, n, C.byref(N), C.byref(nnz)))
    indptr = np.empty(N.value + 1, dtype=np.int64)
    indices = np.empty(nnz.value, dtype=np.int32)
    data = np.empty(nnz.value, dtype=np.float64)
    _lib.check(L.mamg_gen_bidomain(dim, n, float(gamma), float(kappa1), float(kappa2),
                                   _lib.ptr(indptr, C.c_int64), _lib.ptr(indices, C.c_int32),
                                   _lib.ptr(data, C.c_double)))
    return System(indptr, indices, data, int(N.value), int(N.value) // 2, dim, n, float(gamma))


def seeded_rhs(N: int, seed: int = 1234) -> np.ndarray:
    """uniform(-1, 1) fp64, numpy default_rng(seed)."""
    return np.random.default_rng(seed).uniform(-1.0, 1.0, N)
