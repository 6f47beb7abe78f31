"""numpy restatement of the bidomain manufactured solutions -- TEST
INFRASTRUCTURE ONLY (checks csrc/mms.cpp, which the drivers use): load
vector, Dirichlet lifting and H1 errors on the generator's P1 meshes.

The reference solves its bidomain systems against a manufactured solution and
reports the H1 error of both fields with its convergence rate
(src/bidomain_2d.py:7-49 setup_mms, :51-99 get_system, :239-256 errornorm /
rates; src/bidomain_3d.py:7-49, :85-200).  Restated here:

    -div(k1 grad u1) + g (u1 - u2) = f1,  -div(k2 grad u2) + g (u2 - u1) = f2
    2-D: u1 = cos(pi (x + y)),      u2 = sin(pi (x - y))
    3-D: u1 = cos(pi (x + y + 2z)), u2 = sin(pi (x - y + z))

i.e. u1 = cos(pi a.x), u2 = sin(pi c.x), so f1 = k1 pi^2 |a|^2 u1 + g (u1 - u2)
and f2 = k2 pi^2 |c|^2 u2 + g (u2 - u1).  Boundary conditions
(src/bidomain_2d.py:70-96, tags src/utils.py:149-182): Dirichlet u = exact on
tags 1, 2 (x = 0, 1 in 2-D; z = 0, 1 in 3-D), the full flux on the other
faces (L += -(sigma . n, v)_ds with sigma = -k grad u).  The Dirichlet rows are
eliminated symmetrically with a unit diagonal (the generator's matrix,
problems.bidomain): b = F - A[:, D] g off D, b = g on D.

Integrals use collapsed (Duffy) Gauss-Legendre rules on every Kuhn simplex of
dolfin's structured mesh, so the load vector and the error are quadratures of
the exact functions; FEniCS interpolates them into P4 / P2 first
(ulfy degree 4, errornorm degree_rise 1).  Both converge at the same rates;
values agree to the quadrature error, not bitwise (dolfin is absent).
"""
from __future__ import annotations

import itertools

import math

import numpy as np

from mamg_oracle import _K_PATH   # the oracle's own generator (not the product's problems.py)


def _mass_loc(d: int, meas: float) -> np.ndarray:
    """P1 mass matrix of a d-simplex of measure meas: meas/((d+1)(d+2)) (1 + I)."""
    return meas / ((d + 1) * (d + 2)) * (np.ones((d + 1, d + 1)) + np.eye(d + 1))


def _assemble(simplices, index, nv, Kloc, Mloc):
    """Element matrices summed into CSR (K, M) over the vertex numbering `index`."""
    import scipy.sparse as sp
    rows, cols, kv, mv = [], [], [], []
    for verts in simplices:
        ids = [index(v) for v in verts]
        for a in range(len(ids)):
            for b in range(len(ids)):
                rows.append(ids[a])
                cols.append(ids[b])
                kv.append(np.full(len(ids[a]), Kloc[a, b]))
                mv.append(np.full(len(ids[a]), Mloc[a, b]))
    r, c = np.concatenate(rows), np.concatenate(cols)
    K = sp.coo_matrix((np.concatenate(kv), (r, c)), shape=(nv, nv)).tocsr()
    M = sp.coo_matrix((np.concatenate(mv), (r, c)), shape=(nv, nv)).tocsr()
    K.sort_indices()
    M.sort_indices()
    return K, M

_WAVE = {2: (np.array([1.0, 1.0]), np.array([1.0, -1.0])),
         3: (np.array([1.0, 1.0, 2.0]), np.array([1.0, -1.0, 1.0]))}
# Dirichlet axis (tags 1, 2) and the flux axes (tags 3, 4) per dimension
_DIRICHLET_AXIS = {2: 0, 3: 2}
_NEUMANN_AXES = {2: (1,), 3: (0, 1)}


class Exact:
    """u1, u2, their gradients and the loads f1, f2 for kappa1, kappa2, gamma."""

    def __init__(self, dim: int, kappa1: float, kappa2: float, gamma: float):
        self.dim = dim
        self.a, self.c = _WAVE[dim]
        self.k1, self.k2, self.g = float(kappa1), float(kappa2), float(gamma)

    def u(self, X):
        pa, pc = np.pi * (X @ self.a), np.pi * (X @ self.c)
        return np.cos(pa), np.sin(pc)

    def grad(self, X):
        pa, pc = np.pi * (X @ self.a), np.pi * (X @ self.c)
        return (-np.pi * np.sin(pa)[:, None] * self.a[None, :],
                np.pi * np.cos(pc)[:, None] * self.c[None, :])

    def f(self, X):
        u1, u2 = self.u(X)
        f1 = self.k1 * np.pi ** 2 * (self.a @ self.a) * u1 + self.g * (u1 - u2)
        f2 = self.k2 * np.pi ** 2 * (self.c @ self.c) * u2 + self.g * (u2 - u1)
        return f1, f2


def simplex_rule(d: int, m: int = 3):
    """Collapsed Gauss-Legendre rule on the reference d-simplex (d <= 3):
    barycentric coordinates [npts, d+1] and weights summing to 1/d!."""
    t, w = np.polynomial.legendre.leggauss(m)
    t, w = 0.5 * (t + 1.0), 0.5 * w
    pts, wts = [], []
    for idx in itertools.product(range(m), repeat=d):
        u = [t[i] for i in idx]
        wt = float(np.prod([w[i] for i in idx]))
        x, scale = [], 1.0
        for k in range(d):            # x_k = u_k prod_{j<k} (1 - u_j)
            x.append(u[k] * scale)
            if k < d - 1:
                wt *= (1.0 - u[k]) ** (d - 1 - k)
            scale *= 1.0 - u[k]
        pts.append([1.0 - sum(x)] + x)
        wts.append(wt)
    return np.array(pts), np.array(wts)


def _paths(dim: int, cells: np.ndarray):
    """(perm, [vertex lattice coords]) of every Kuhn path simplex of the cells."""
    for perm in itertools.permutations(range(dim)):
        verts = [cells]
        cur = cells
        for ax in perm:
            cur = cur.copy()
            cur[:, ax] += 1
            verts.append(cur)
        yield perm, verts


def _lattice(shape):
    g = np.meshgrid(*[np.arange(s) for s in shape], indexing='ij')
    return np.stack([x.ravel() for x in g], axis=1).astype(np.int64)


class BidomainMMS:
    """Manufactured-solution data of problems.bidomain(dim, n, gamma, kappa1,
    kappa2) in its vertex numbering (x fastest; u1 dofs then u2 dofs)."""

    CHUNK = 1 << 20   # cells per vectorised pass

    def __init__(self, dim: int, n: int, gamma: float, kappa1: float = 2.0, kappa2: float = 3.0,
                 qorder: int = 3):
        if dim not in (2, 3):
            raise ValueError('dim must be 2 or 3')
        self.dim, self.n = dim, n
        self.h = 1.0 / n
        self.nv = (n + 1) ** dim
        self.ex = Exact(dim, kappa1, kappa2, gamma)
        self.lam, self.w = simplex_rule(dim, qorder)
        self.flam, self.fw = simplex_rule(dim - 1, qorder)
        self.stride = (n + 1) ** np.arange(dim)

    def cell_chunks(self):
        """lower-corner lattice coordinates of all cells, CHUNK at a time"""
        nc = self.n ** self.dim
        for c0 in range(0, nc, self.CHUNK):
            ids = np.arange(c0, min(nc, c0 + self.CHUNK), dtype=np.int64)
            yield (ids[:, None] // (self.n ** np.arange(self.dim))[None, :]) % self.n

    def index(self, V):
        return V @ self.stride

    def coords(self, ids: np.ndarray) -> np.ndarray:
        """lattice coordinates of vertex ids"""
        return (np.asarray(ids)[:, None] // self.stride[None, :]) % (self.n + 1)

    def dirichlet_nodes(self) -> np.ndarray:
        V = self.coords(np.arange(self.nv))
        ax = _DIRICHLET_AXIS[self.dim]
        return np.flatnonzero((V[:, ax] == 0) | (V[:, ax] == self.n))

    def load(self) -> np.ndarray:
        """F = [(f1, v); (f2, v)] + the flux terms on tags 3, 4 (no BCs yet)."""
        d, h, nv = self.dim, self.h, self.nv
        F = np.zeros(2 * nv)
        for _, verts in (pv for c in self.cell_chunks() for pv in _paths(d, c)):
            X = [v * h for v in verts]
            ids = [self.index(v) for v in verts]
            for q in range(len(self.w)):
                x = sum(self.lam[q, k] * X[k] for k in range(d + 1))
                f1, f2 = self.ex.f(x)
                wq = self.w[q] * h ** d
                for k in range(d + 1):
                    F[:nv] += np.bincount(ids[k], wq * self.lam[q, k] * f1, minlength=nv)
                    F[nv:] += np.bincount(ids[k], wq * self.lam[q, k] * f2, minlength=nv)
        for ax in _NEUMANN_AXES[d]:
            other = [a for a in range(d) if a != ax]
            fcells = _lattice([self.n] * (d - 1))
            for side in (0, 1):
                normal = np.zeros(d)
                normal[ax] = 1.0 if side else -1.0
                for _, fv in _paths(d - 1, fcells):
                    verts = []
                    for v in fv:      # embed the facet vertex in the face x_ax = side
                        V = np.zeros((len(v), d), np.int64)
                        V[:, other] = v
                        V[:, ax] = side * self.n
                        verts.append(V)
                    X = [v * h for v in verts]
                    ids = [self.index(v) for v in verts]
                    for q in range(len(self.fw)):
                        x = sum(self.flam[q, k] * X[k] for k in range(d))
                        g1, g2 = self.ex.grad(x)
                        # -(sigma . n) = k grad u . n
                        t1 = self.ex.k1 * (g1 @ normal)
                        t2 = self.ex.k2 * (g2 @ normal)
                        wq = self.fw[q] * h ** (d - 1)
                        for k in range(d):
                            F[:nv] += np.bincount(ids[k], wq * self.flam[q, k] * t1, minlength=nv)
                            F[nv:] += np.bincount(ids[k], wq * self.flam[q, k] * t2, minlength=nv)
        return F

    def full_matrix(self, cells=None):
        """The bidomain matrix before the Dirichlet elimination, summed over the
        given cells (default all)."""
        import scipy.sparse as sp
        d, h = self.dim, self.h
        Kloc = _K_PATH[d].astype(np.float64) / math.factorial(d) * h ** (d - 2)   # path-simplex stiffness
        Mloc = _mass_loc(d, h ** d / math.factorial(d))
        if cells is None:
            cells = _lattice([self.n] * d)
        simp = [verts for _, verts in _paths(d, cells)]
        K, M = _assemble(simp, self.index, self.nv, Kloc, Mloc)
        e = self.ex
        A = sp.bmat([[e.k1 * K + e.g * M, -e.g * M], [-e.g * M, e.k2 * K + e.g * M]], format='csr')
        A.sort_indices()
        return A

    def rhs(self) -> np.ndarray:
        """b of the eliminated system: F - A[:, D] g off the Dirichlet rows, g on them."""
        F = self.load()
        nv = self.nv
        Dn = self.dirichlet_nodes()
        D = np.concatenate([Dn, nv + Dn])
        V = self.coords(Dn) * self.h
        u1, u2 = self.ex.u(V)
        g = np.zeros(2 * nv)
        g[Dn], g[nv + Dn] = u1, u2
        # A[:, D] g only involves the cells of the two Dirichlet layers
        cells = _lattice([self.n] * self.dim)
        ax = _DIRICHLET_AXIS[self.dim]
        cells = cells[(cells[:, ax] == 0) | (cells[:, ax] == self.n - 1)]
        A = self.full_matrix(cells)
        b = F - A @ g
        b[D] = g[D]
        return b

    def h1_errors(self, x: np.ndarray):
        """(|u1 - u1h|_H1, |u2 - u2h|_H1), full H1 norm (errornorm 'H1')."""
        d, h, nv = self.dim, self.h, self.nv
        x = np.asarray(x, dtype=np.float64)
        e2 = np.zeros(2)
        for perm, verts in (pv for c in self.cell_chunks() for pv in _paths(d, c)):
            X = [v * h for v in verts]
            ids = [self.index(v) for v in verts]
            for f, off in ((0, 0), (1, nv)):
                uk = [x[off + i] for i in ids]
                gh = np.zeros((len(ids[0]), d))   # P1 gradient along the path's steps
                for j, ax in enumerate(perm):
                    gh[:, ax] = (uk[j + 1] - uk[j]) / h
                acc = np.zeros(len(ids[0]))
                for q in range(len(self.w)):
                    xq = sum(self.lam[q, k] * X[k] for k in range(d + 1))
                    u = self.ex.u(xq)[f]
                    g = self.ex.grad(xq)[f]
                    uh = sum(self.lam[q, k] * uk[k] for k in range(d + 1))
                    acc += self.w[q] * ((u - uh) ** 2 + ((g - gh) ** 2).sum(axis=1))
                e2[f] += acc.sum() * h ** d
        return float(np.sqrt(e2[0])), float(np.sqrt(e2[1]))


def rates(errors, hs):
    """log(e_k / e_{k-1}) / log(h_k / h_{k-1}) (nan first), src/bidomain_2d.py:236-239."""
    errors, hs = np.asarray(errors, float), np.asarray(hs, float)
    out = np.full(errors.shape, np.nan)
    if len(errors) > 1:
        out[1:] = np.log(errors[1:] / errors[:-1]) / np.log(hs[1:] / hs[:-1])[:, None] \
            if errors.ndim == 2 else np.log(errors[1:] / errors[:-1]) / np.log(hs[1:] / hs[:-1])
    return out
