"""CPU restatement of the reference's OWN metric_mono algorithm -- TEST
INFRASTRUCTURE ONLY (never imported by the product).

PARITY STATUS: parity unpinned.  The reference selects HAZmath's metric AMG
with ``parameters_metric_schwarz`` (/root/reference/src/amg_parameters.py:67-89,
selected at src/bidomain_3d.py:144-145):
    AMG_type UA_AMG (:68), cycle_type W_CYCLE (:69), max_levels 20, maxit 1,
    smoother SMOOTHER_SGS (:72), presmooth/postsmooth 1 (:74-75),
    coarse_dof 100 (:76), coarse_solver UMFPACK (:77), coarse_scaling ON (:78),
    aggregation_type HEM (:79), strong_coupled 0.1 (:80),
    Schwarz_levels 1, mmsize 100, maxlvl 1, SCHWARZ_SYMMETRIC (:83-86),
    seeds = idofs (src/utils.py:84-86).
HAZmath's source is not in /root/reference and not installable here, so every
component below is a restatement of its published algorithm family [ext,
recalled], not a pinned copy:
  * HEM: greedy heavy-edge matching over the strength graph
    (|a_ij| >= theta sqrt(|a_ii a_jj|)), vertices in index order, each
    unmatched vertex pairs with its heaviest unmatched strong neighbour (ties:
    smallest index); unmatched vertices are singletons.  Two passes per level
    (the second matches the pairs on their Galerkin graph), so aggregates hold
    up to 4 dofs -- one pass alone coarsens by < 2 and the W-cycle's work
    then grows without bound with the number of levels;
  * UA: piecewise-constant P, Galerkin A_c = P^T A P;
  * SGS: forward then backward Gauss-Seidel (exact triangular solves);
  * level-0 symmetric multiplicative Schwarz: one block per seed = the seed and
    its Schwarz_maxlvl-ring in A's graph (BFS, at most Schwarz_mmsize dofs),
    exact block solves, forward then backward over the seeds; dofs in no block
    get Gauss-Seidel (src/utils.py:84: "the rest the GS smoother");
  * W-cycle (the coarse problem visited twice), coarse-grid correction scaled
    by alpha = <r, Pe> / <A Pe, Pe> when coarse_scaling is ON;
  * coarsest: dense direct solve.
Its purpose is to quantify the iteration-count gap between the reference's
sequential algorithm and the GPU profile, not to pin
the product.
"""
from __future__ import annotations

import dataclasses
from collections import deque

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp
from scipy.sparse.linalg import spsolve_triangular


@dataclasses.dataclass
class RefParams:
    cycle_type: str = 'W'
    max_levels: int = 20
    coarse_dof: int = 100
    coarse_scaling: bool = True
    strong_coupled: float = 0.1
    Schwarz_levels: int = 1
    Schwarz_mmsize: int = 100
    Schwarz_maxlvl: int = 1
    presmooth_iter: int = 1
    postsmooth_iter: int = 1
    hem_passes: int = 2          # matching passes per level (aggregates of <= 2^passes)


def hem_aggregate(A: sp.csr_matrix, theta: float):
    """one greedy heavy-edge matching pass -> (agg[n], nagg)"""
    n = A.shape[0]
    d = np.abs(A.diagonal())
    agg = np.full(n, -1, dtype=np.int64)
    nagg = 0
    ip, ix, dv = A.indptr, A.indices, np.abs(A.data)
    for i in range(n):
        if agg[i] >= 0:
            continue
        best, bw = -1, -1.0
        for k in range(ip[i], ip[i + 1]):
            j = ix[k]
            if j == i or agg[j] >= 0:
                continue
            w = dv[k]
            if w < theta * np.sqrt(d[i] * d[j]) or w == 0.0:
                continue
            if w > bw or (w == bw and j < best):
                best, bw = j, w
        agg[i] = nagg
        if best >= 0:
            agg[best] = nagg
        nagg += 1
    return agg, nagg


def schwarz_blocks(A: sp.csr_matrix, seeds, maxlvl: int, mmsize: int):
    """seed + maxlvl-ring (BFS order, neighbours ascending), <= mmsize dofs"""
    ip, ix = A.indptr, A.indices
    blocks = []
    for s in seeds:
        seen = {int(s)}
        order = [int(s)]
        q = deque([(int(s), 0)])
        while q and len(order) < mmsize:
            v, lv = q.popleft()
            if lv == maxlvl:
                continue
            for j in sorted(ix[ip[v]:ip[v + 1]]):
                if j not in seen:
                    seen.add(int(j))
                    order.append(int(j))
                    q.append((int(j), lv + 1))
                    if len(order) >= mmsize:
                        break
        blocks.append(np.array(sorted(order), dtype=np.int64))
    return blocks


class RefLevel:
    def __init__(self, A):
        self.A = A.tocsr()
        self.L = sp.tril(self.A, format='csr')
        self.U = sp.triu(self.A, format='csr')
        self.P = None
        self.blocks = None
        self.block_inv = None
        self.rest = None
        self.Ainv = None


class RefHierarchy:
    def __init__(self, A, idofs, p: RefParams):
        self.p = p
        self.levels = []
        cur = A.tocsr()
        cur.sort_indices()
        for l in range(p.max_levels):
            lev = RefLevel(cur)
            self.levels.append(lev)
            n = cur.shape[0]
            if n <= p.coarse_dof or l == p.max_levels - 1:
                lev.Ainv = sla.lu_factor(cur.toarray())
                break
            agg, nagg = hem_aggregate(cur, p.strong_coupled)
            for _ in range(p.hem_passes - 1):       # aggregates of matched pairs
                T1 = sp.csr_matrix((np.ones(n), (np.arange(n), agg)), shape=(n, nagg))
                A1 = (T1.T @ cur @ T1).tocsr()
                A1.sort_indices()
                a2, nagg = hem_aggregate(A1, p.strong_coupled)
                agg = a2[agg]
            if nagg > 0.9 * n:                  # coarsening stalled: solve directly here
                lev.Ainv = sla.lu_factor(cur.toarray())
                break
            lev.P = sp.csr_matrix((np.ones(n), (np.arange(n), agg)), shape=(n, nagg))
            if l < p.Schwarz_levels and idofs is not None and len(idofs):
                lev.blocks = schwarz_blocks(cur, idofs, p.Schwarz_maxlvl, p.Schwarz_mmsize)
                lev.block_rows = [cur[b] for b in lev.blocks]
                lev.block_inv = [sla.lu_factor(R[:, b].toarray()) for R, b in zip(lev.block_rows, lev.blocks)]
                covered = np.zeros(n, bool)
                for b in lev.blocks:
                    covered[b] = True
                lev.rest = np.flatnonzero(~covered)
                Ar = cur[lev.rest][:, lev.rest]
                lev.Lr = sp.tril(Ar, format='csr')
                lev.Ur = sp.triu(Ar, format='csr')
            cur = (lev.P.T @ cur @ lev.P).tocsr()
            cur.sort_indices()

    # -- smoothers ------------------------------------------------------------
    @staticmethod
    def _gs(lev, x, b, forward):
        r = b - lev.A @ x
        T = lev.L if forward else lev.U
        return x + spsolve_triangular(T, r, lower=forward)

    def _schwarz(self, lev, x, b, forward):
        order = range(len(lev.blocks)) if forward else range(len(lev.blocks) - 1, -1, -1)
        A = lev.A
        for k in order:
            blk = lev.blocks[k]
            rb = b[blk] - lev.block_rows[k] @ x
            x[blk] += sla.lu_solve(lev.block_inv[k], rb, check_finite=False)
        if len(lev.rest):                        # Gauss-Seidel on the uncovered dofs
            rr = (b - A @ x)[lev.rest]
            T = lev.Lr if forward else lev.Ur
            x[lev.rest] += spsolve_triangular(T, rr, lower=forward)
        return x

    def _smooth(self, lev, x, b, pre):
        # symmetric: pre = forward then backward, post = the same (SGS / symmetric Schwarz)
        for fwd in (True, False):
            if lev.blocks is not None:
                x = self._schwarz(lev, x, b, fwd)
            else:
                x = self._gs(lev, x, b, fwd)
        return x

    # -- cycle ----------------------------------------------------------------
    def cycle(self, l, b):
        lev = self.levels[l]
        if lev.Ainv is not None:
            return sla.lu_solve(lev.Ainv, b)
        x = np.zeros_like(b)
        for _ in range(self.p.presmooth_iter):
            x = self._smooth(lev, x, b, True)
        visits = 2 if self.p.cycle_type == 'W' else 1
        for _ in range(visits):
            r = b - lev.A @ x
            e = lev.P @ self.cycle(l + 1, lev.P.T @ r)
            alpha = 1.0
            if self.p.coarse_scaling:
                Ae = lev.A @ e
                den = float(Ae @ e)
                alpha = float(r @ e) / den if den > 0 else 1.0
            x = x + alpha * e
        for _ in range(self.p.postsmooth_iter):
            x = self._smooth(lev, x, b, False)
        return x

    def apply(self, r):
        return self.cycle(0, np.asarray(r, dtype=np.float64))

    __call__ = apply
