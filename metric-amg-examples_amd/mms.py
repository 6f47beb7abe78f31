"""Manufactured solutions of the drivers (right-hand sides and H1 errors).

Bidomain (src/bidomain_2d.py:7-99, src/bidomain_3d.py:7-49): csrc/mms.cpp
through the C-ABI (``problems.bidomain_mms_rhs`` / ``bidomain_mms_errors``,
re-exported here).

EMI (src/emi_2d.py:8-128, src/emi_3d.py:8-55), restated here in numpy on the
split meshes of ``problems.emi``:

    -div(k_i grad u_i) = f_i in Omega_i,  Omega_1 = {x_d > 1/2}, Omega_2 = {x_d < 1/2}
    2-D: u1 = cos(pi (x + y)),      u2 = sin(pi (x + y))
    3-D: u1 = cos(pi (x + y + 2z)), u2 = sin(pi (x + y - z))
    sigma_i = k_i grad u_i;  on Gamma = {x_d = 1/2}: n1 = -e_d, n2 = +e_d,
    g_n = -sigma1.n1 - sigma2.n2,  g_r = -sigma1.n1 - gamma (u1 - u2)
    L1 = (f1, v1) + (sigma1.n, v1)_sides - (g_r, v1)_Gamma
    L2 = (f2, v2) + (sigma2.n, v2)_sides - (g_n, v2)_Gamma + (g_r, v2)_Gamma
    Dirichlet: u1 on x_d = 1 (tag 3), u2 on x_d = 0 (tag 6), lifted and
    eliminated as problems.emi does.

Integrals: collapsed Gauss-Legendre (3 points per direction) on the Kuhn
simplices, as csrc/mms.cpp.  The EMI drivers check these by their H1 rate
(tests/test_mms.py, direct solves).
"""
from __future__ import annotations

import itertools

import numpy as np

from . import problems
from .problems import bidomain_mms_errors, bidomain_mms_rhs  # noqa: F401  (re-export)

_EMI_WAVE = {2: (np.array([1.0, 1.0]), np.array([1.0, 1.0])),
             3: (np.array([1.0, 1.0, 2.0]), np.array([1.0, 1.0, -1.0]))}


def simplex_rule(d: int, m: int = 3):
    """Collapsed Gauss-Legendre rule on the reference d-simplex: barycentric
    coordinates [npts, d+1], weights summing to 1/d!."""
    t, w = np.polynomial.legendre.leggauss(m)
    t, w = 0.5 * (t + 1.0), 0.5 * w
    pts, wts = [], []
    for idx in itertools.product(range(m), repeat=d):
        wt, scale, x = float(np.prod([w[i] for i in idx])), 1.0, []
        for k, i in enumerate(idx):      # x_k = u_k prod_{j<k} (1 - u_j)
            x.append(t[i] * scale)
            if k < d - 1:
                wt *= (1.0 - t[i]) ** (d - 1 - k)
            scale *= 1.0 - t[i]
        pts.append([1.0 - sum(x)] + x)
        wts.append(wt)
    return np.array(pts), np.array(wts)


def _paths(dim: int, cells: np.ndarray):
    """(perm, vertex lattice coords) of the Kuhn path simplices of the cells
    (problems._simplices' order)."""
    for perm in itertools.permutations(range(dim)):
        verts, cur = [cells], cells
        for ax in perm:
            cur = cur.copy()
            cur[:, ax] += 1
            verts.append(cur)
        yield perm, verts


def _lattice(shape):
    g = np.meshgrid(*[np.arange(s) for s in shape], indexing='ij')
    return np.stack([x.ravel() for x in g], axis=1).astype(np.int64)


class EmiMMS:
    """Manufactured-solution data of problems.emi(dim, n, gamma, kappa1, kappa2)."""

    def __init__(self, dim: int, n: int, gamma: float, kappa1: float = 2.0, kappa2: float = 3.0):
        if dim not in (2, 3) or n < 4 or n % 2:
            raise ValueError('dim must be 2 or 3, n even and >= 4')
        self.dim, self.n, self.m = dim, n, n // 2
        self.h = 1.0 / n
        self.k = (float(kappa1), float(kappa2))
        self.g = float(gamma)
        self.a, self.c = _EMI_WAVE[dim]
        self.nv = (n + 1) ** (dim - 1) * (self.m + 1)
        self.rule = simplex_rule(dim)
        self.frule = simplex_rule(dim - 1)

    # exact solution ---------------------------------------------------------
    def u(self, X):
        return np.cos(np.pi * (X @ self.a)), np.sin(np.pi * (X @ self.c))

    def grad(self, X):
        return (-np.pi * np.sin(np.pi * (X @ self.a))[:, None] * self.a,
                np.pi * np.cos(np.pi * (X @ self.c))[:, None] * self.c)

    def f(self, X):
        u1, u2 = self.u(X)
        return (self.k[0] * np.pi ** 2 * (self.a @ self.a) * u1,
                self.k[1] * np.pi ** 2 * (self.c @ self.c) * u2)

    # assembly helpers -------------------------------------------------------
    def _volume(self, top: bool, fn, out):
        """out += (fn(x), phi_i) over the half's simplices"""
        d, h = self.dim, self.h
        cells, index = problems.emi_half(d, self.n, top)
        lam, w = self.rule
        for _, verts in _paths(d, cells):
            X = [v * h for v in verts]
            ids = [index(v) for v in verts]
            for q in range(len(w)):
                val = fn(sum(lam[q, k] * X[k] for k in range(d + 1)))
                for k in range(d + 1):
                    out += np.bincount(ids[k], w[q] * h ** d * lam[q, k] * val, minlength=self.nv)

    def _facets(self, top: bool, axis: int, level: int, layers):
        """(X, ids) of the (d-1)-simplices of the plane x_axis = level h, over
        the cell layers `layers` of the interface axis (all if axis is it)"""
        d, n = self.dim, self.n
        other = [a for a in range(d) if a != axis]
        shape = [n if a != d - 1 else len(layers) for a in other]
        fc = _lattice(shape)
        if d - 1 in other:
            j = other.index(d - 1)
            fc[:, j] = np.asarray(layers)[fc[:, j]]
        _, index = problems.emi_half(d, n, top)
        for _, fv in _paths(d - 1, fc):
            verts = []
            for v in fv:
                V = np.zeros((len(v), d), np.int64)
                V[:, other] = v
                V[:, axis] = level
                verts.append(V)
            yield [v * self.h for v in verts], [index(v) for v in verts]

    def _surface(self, facets, fn, out):
        d = self.dim
        lam, w = self.frule
        for X, ids in facets:
            for q in range(len(w)):
                val = fn(sum(lam[q, k] * X[k] for k in range(d)))
                for k in range(d):
                    out += np.bincount(ids[k], w[q] * self.h ** (d - 1) * lam[q, k] * val, minlength=self.nv)

    def load(self):
        """[L1, L2] before the Dirichlet rows (src/emi_2d.py:99-121)."""
        d, n, m = self.dim, self.n, self.m
        k1, k2, g, ax = self.k[0], self.k[1], self.g, self.dim - 1
        L1, L2 = np.zeros(self.nv), np.zeros(self.nv)
        self._volume(True, lambda X: self.f(X)[0], L1)
        self._volume(False, lambda X: self.f(X)[1], L2)
        # full flux on the side faces of each half: (sigma_i . n, v_i)
        for a in range(d - 1):
            for side in (0, 1):
                sgn = 1.0 if side else -1.0
                self._surface(self._facets(True, a, side * n, range(m, n)),
                              lambda X: sgn * k1 * self.grad(X)[0][:, a], L1)
                self._surface(self._facets(False, a, side * n, range(0, m)),
                              lambda X: sgn * k2 * self.grad(X)[1][:, a], L2)
        # interface terms; -sigma1.n1 = k1 du1/dx_d, -sigma2.n2 = -k2 du2/dx_d

        def g_r(X):
            u1, u2 = self.u(X)
            return k1 * self.grad(X)[0][:, ax] - g * (u1 - u2)

        def g_n(X):
            g1, g2 = self.grad(X)
            return k1 * g1[:, ax] - k2 * g2[:, ax]
        self._surface(self._facets(True, ax, m, None), lambda X: -g_r(X), L1)
        self._surface(self._facets(False, ax, m, None), lambda X: g_r(X) - g_n(X), L2)
        return L1, L2

    def dirichlet(self):
        """outer-layer dofs (x_d = 1 for u1, x_d = 0 for u2) and their values"""
        d, n, m = self.dim, self.n, self.m
        ng = (n + 1) ** (d - 1)
        dofs = np.arange(self.nv - ng, self.nv)
        V = _lattice([n + 1] * (d - 1))[:, ::-1]          # lattice order, axis 0 fastest
        X1 = np.concatenate([V, np.full((ng, 1), n)], axis=1) * self.h
        X2 = np.concatenate([V, np.zeros((ng, 1), np.int64)], axis=1) * self.h
        return dofs, self.u(X1)[0], self.u(X2)[1]

    def rhs(self):
        """[b1, b2] of problems.emi's (eliminated) block system."""
        import scipy.sparse as sp
        L1, L2 = self.load()
        d, h = self.dim, self.h
        Kloc = problems._PATH_K[d] * (h if d == 3 else 1.0)
        Mloc = problems._mass_loc(d, h ** d / (2 if d == 2 else 6))
        dofs, g1, g2 = self.dirichlet()
        for top, L, gv, kap in ((True, L1, g1, self.k[0]), (False, L2, g2, self.k[1])):
            cells, index = problems.emi_half(d, self.n, top)
            K = problems._assemble(problems._simplices(cells, d), index, self.nv, Kloc, Mloc)[0]
            gfull = np.zeros(self.nv)
            gfull[dofs] = gv
            L -= kap * (K @ gfull)      # the coupling blocks never reach the outer layers
            L[dofs] = gv
        return [L1, L2]

    def h1_errors(self, x1, x2):
        """(|u1 - u1h|_H1(Omega_1), |u2 - u2h|_H1(Omega_2))"""
        d, h = self.dim, self.h
        lam, w = self.rule
        out = []
        for top, x, f in ((True, x1, 0), (False, x2, 1)):
            cells, index = problems.emi_half(d, self.n, top)
            e2 = 0.0
            for perm, verts in _paths(d, cells):
                X = [v * h for v in verts]
                uk = [x[index(v)] for v in verts]
                gh = np.zeros((len(cells), d))
                for j, ax in enumerate(perm):
                    gh[:, ax] = (uk[j + 1] - uk[j]) / h
                acc = np.zeros(len(cells))
                for q in range(len(w)):
                    xq = sum(lam[q, k] * X[k] for k in range(d + 1))
                    u = self.u(xq)[f]
                    gq = self.grad(xq)[f]
                    uh = sum(lam[q, k] * uk[k] for k in range(d + 1))
                    acc += w[q] * ((u - uh) ** 2 + ((gq - gh) ** 2).sum(axis=1))
                e2 += acc.sum() * h ** d
            out.append(float(np.sqrt(e2)))
        return tuple(out)


def emi_mms_rhs(dim: int, n: int, gamma: float, kappa1: float = 2.0, kappa2: float = 3.0):
    """[b1, b2] of problems.emi(dim, n, ...) for the reference's manufactured solution."""
    return EmiMMS(dim, n, gamma, kappa1, kappa2).rhs()


def emi_mms_errors(dim: int, n: int, x, gamma: float, kappa1: float = 2.0, kappa2: float = 3.0):
    """H1 errors of a block solution x = [x1, x2] (or the monolithic vector)."""
    P = EmiMMS(dim, n, gamma, kappa1, kappa2)
    if not isinstance(x, (list, tuple)):
        x = np.asarray(x)
        x = [x[:P.nv], x[P.nv:]]
    return P.h1_errors(np.asarray(x[0], np.float64), np.asarray(x[1], np.float64))
