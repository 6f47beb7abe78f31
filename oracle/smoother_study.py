"""Smoother / cycle ablation study -- TEST INFRASTRUCTURE ONLY.

Which GPU-parallel components close the PCG iteration gap between the GPU
profile and the reference's metric_mono (ref_profile.py)?
Every variant below is deterministic and round-synchronous, so a HIP kernel
can reproduce it: multicolor node-block SGS (colours from a hash-priority
Jones-Plassmann colouring), coarse-grid correction scaling computed on the
coarse level (alpha = <b_c, e>/<A_c e, e>), W-cycle.

    python oracle/smoother_study.py [dim n gamma ...]
"""
from __future__ import annotations

import itertools
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import mamg_oracle as mo            # noqa: E402
from ref_profile import RefHierarchy, RefParams   # noqa: E402


def node_graph(A, nf):
    n = A.shape[0]
    nv = n // nf
    r = np.repeat(np.arange(n), np.diff(A.indptr)) % nv
    c = A.indices % nv
    G = sp.csr_matrix((np.ones(len(r)), (r, c)), shape=(nv, nv))
    G = ((G + G.T) != 0).astype(np.int8).tocsr()
    G.setdiag(0)
    G.eliminate_zeros()
    G.sort_indices()
    return G


def jp_colour(G, level=0):
    """Round-synchronous Jones-Plassmann: an uncoloured node whose key
    (hash prio, index) beats every uncoloured neighbour takes the smallest
    colour no coloured neighbour holds."""
    nv = G.shape[0]
    col = np.full(nv, -1, np.int64)
    pr = (mo.hash32(np.arange(nv), 1000 + level).astype(np.uint64) << np.uint64(32)) | np.arange(nv, dtype=np.uint64)
    ip, ix = G.indptr, G.indices
    rr = np.repeat(np.arange(nv), np.diff(ip))
    while (col < 0).any():
        unc = col < 0
        key = np.where(unc, pr, np.uint64(0))
        nbmax = np.zeros(nv, np.uint64)
        m = unc[ix]
        np.maximum.at(nbmax, rr[m], key[ix[m]])
        win = unc & (key > nbmax)
        mask = np.zeros(nv, np.uint64)
        cm = (~unc)[ix] & win[rr]
        np.bitwise_or.at(mask, rr[cm], np.left_shift(np.uint64(1), col[ix[cm]].astype(np.uint64)))
        w = np.flatnonzero(win)
        free = (~mask[w]) & (mask[w] + np.uint64(1))
        col[w] = np.log2(free.astype(np.float64)).astype(np.int64)
    return col


class Study:
    def __init__(self, A, idofs, cycle='V', smoother='bjac', scaling=False, amg='SA',
                 omega=1.0, nsweep=1, l0=None, **pkw):
        p = mo.Params(num_functions=2, AMG_type=amg, **pkw)
        self.h = mo.setup(A, p, idofs=idofs)
        self.cycle_type = cycle
        self.smoother = smoother
        self.l0 = l0 or smoother
        self.scaling = scaling
        self.omega = omega
        self.nsweep = nsweep
        self.lv = []
        for l, lev in enumerate(self.h.levels):
            d = {}
            if lev.Ainv is None:
                n = lev.A.shape[0]
                nv = n // 2
                G = node_graph(lev.A, 2)
                colv = jp_colour(G, l)
                bid, nb = mo.node_blocks(n, 2)
                Dinv = mo.block_inverse_csr(lev.A, bid, nb)
                cols = np.tile(colv, 2)
                d['ncol'] = int(colv.max()) + 1
                d['rows'] = [np.flatnonzero(cols == c) for c in range(d['ncol'])]
                d['Arows'] = [lev.A[r] for r in d['rows']]
                d['Dinv'] = [Dinv[r][:, r] for r in d['rows']]
                d['full_Dinv'] = Dinv
            self.lv.append(d)
        self.ncolours = [d.get('ncol', 0) for d in self.lv]

    def _mcsgs(self, l, x, b, order):
        d = self.lv[l]
        for c in order:
            rw = d['rows'][c]
            rres = b[rw] - d['Arows'][c] @ x
            x[rw] += self.omega * (d['Dinv'][c] @ rres)
        return x

    def _smooth(self, l, x, b, pre):
        lev = self.h.levels[l]
        kind = self.l0 if l == 0 else self.smoother
        nc = self.lv[l]['ncol']
        for _ in range(self.nsweep):
            if kind == 'bjac':
                x = x + lev.smooth_apply(b - lev.A @ x)
            elif kind == 'mcsgs':
                x = self._mcsgs(l, x, b, range(nc))
                x = self._mcsgs(l, x, b, range(nc - 1, -1, -1))
            elif kind == 'mcgs':      # forward pre, backward post (symmetric cycle)
                x = self._mcsgs(l, x, b, range(nc) if pre else range(nc - 1, -1, -1))
            else:
                raise ValueError(kind)
        return x

    def cycle(self, l, b):
        lev = self.h.levels[l]
        if lev.Ainv is not None:
            return lev.Ainv @ b
        x = self._smooth(l, np.zeros_like(b), b, True)
        nxt = self.h.levels[l + 1]
        visits = 2 if (self.cycle_type == 'W' and nxt.Ainv is None) else 1
        for _ in range(visits):
            r = b - lev.A @ x
            bc = lev.R @ r
            e = self.cycle(l + 1, bc)
            alpha = 1.0
            if self.scaling:
                den = float(e @ (nxt.A @ e))
                alpha = float(bc @ e) / den if den > 0 else 1.0
            x = x + alpha * (lev.P @ e)
        return self._smooth(l, x, b, False)

    def __call__(self, r):
        return self.cycle(0, np.asarray(r, np.float64))


VARIANTS = {
    'bjac_V': dict(),
    'bjac_W': dict(cycle='W'),
    'mcsgs_V': dict(smoother='mcsgs'),
    'mcsgs_V_s': dict(smoother='mcsgs', scaling=True),
    'mcsgs_W': dict(smoother='mcsgs', cycle='W'),
    'mcsgs_W_s': dict(smoother='mcsgs', cycle='W', scaling=True),
    'mcgs_V': dict(smoother='mcgs'),
    'mcgs_V_s': dict(smoother='mcgs', scaling=True),
    'bjac_V_s': dict(scaling=True),
    'UA_mcsgs_W_s': dict(amg='UA', smoother='mcsgs', cycle='W', scaling=True),
}


def run(cases, variants, with_ref=True):
    for dim, n, g in cases:
        s = mo.bidomain_system(dim, n, g)
        A = s['A']
        b = mo.seeded_rhs(A.shape[0])
        out = dict(dim=dim, n=n, N=A.shape[0], gamma=g)
        if with_ref:
            h = RefHierarchy(A, s['idofs'], RefParams())
            out['ref'] = mo.pcg(A, h, b, 1e-8, 500).niters
        for name in variants:
            t0 = time.time()
            st = Study(A, s['idofs'], **VARIANTS[name])
            res = mo.pcg(A, st, b, 1e-8, 500)
            out[name] = res.niters
            out[name + '_ncol'] = st.ncolours[0]
        print(out, flush=True)


if __name__ == '__main__':
    args = sys.argv[1:]
    if args:
        cases = [(int(args[i]), int(args[i + 1]), float(args[i + 2])) for i in range(0, len(args), 3)]
    else:
        cases = [(3, 16, 1.0), (3, 16, 1e6), (3, 16, 1e10), (3, 32, 1e6)]
    run(cases, list(VARIANTS), with_ref=os.environ.get('NOREF') is None)


# ---------------------------------------------------------------------------
# level-0 node-patch Schwarz: patch(I) = both fields of the closed node
# neighbourhood N[I] (= the reference's seed u2_I + 1-ring of A's graph when
# the seeds are the u2 dofs, src/amg_parameters.py:83-86, src/utils.py:84)
# ---------------------------------------------------------------------------
def node_patches(A, nf=2):
    G = node_graph(A, nf)
    nv = G.shape[0]
    pats = []
    for I in range(nv):
        nodes = np.sort(np.r_[I, G.indices[G.indptr[I]:G.indptr[I + 1]]])
        pats.append(np.concatenate([f * nv + nodes for f in range(nf)]))
    return pats, G


def patch_operator(A, pats, dtype=np.float64):
    """S = sum_k R_k^T A_k^-1 R_k (assembled sparse)."""
    A = A.tocsr()
    rows, cols, vals = [], [], []
    for p in pats:
        Ak = A[p][:, p].toarray()
        Ki = np.linalg.inv(Ak).astype(dtype).astype(np.float64)
        rows.append(np.repeat(p, len(p)))
        cols.append(np.tile(p, len(p)))
        vals.append(Ki.ravel())
    S = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=A.shape)
    S.sum_duplicates()
    return S


def power_rho(M, A, iters=30):
    v = mo.hash32(np.arange(A.shape[0]), 5).astype(np.float64) / 4.3e9 - 0.5
    lam = 0.0
    for _ in range(iters):
        w = M @ (A @ v)
        lam = float(np.linalg.norm(w) / np.linalg.norm(v))
        v = w / np.linalg.norm(w)
    return lam


class PatchStudy(Study):
    """level 0: additive ('asm') or multicolour multiplicative ('msm') node-patch
    Schwarz; coarser levels: `smoother` (bjac / mcsgs)."""

    def __init__(self, A, idofs, l0kind='asm', asm_w=None, **kw):
        super().__init__(A, idofs, **kw)
        A0 = self.h.levels[0].A
        self.pats, G = node_patches(A0)
        self.l0kind = l0kind
        if l0kind == 'asm':
            self.S = patch_operator(A0, self.pats)
            rho = power_rho(self.S, A0)
            self.asm_w = asm_w if asm_w is not None else 1.0 / rho
            self.rho = rho
        else:
            # distance-2 colouring of patches (patches of one colour are disjoint and uncoupled)
            G2 = (G @ G + G).astype(bool).astype(np.int8).tocsr()
            G2.setdiag(0)
            G2.eliminate_zeros()
            self.pcol = jp_colour(G2, 77)
            self.npcol = int(self.pcol.max()) + 1
            self.pinv = [np.linalg.inv(A0[p][:, p].toarray()) for p in self.pats]
            self.prow = [A0[p] for p in self.pats]
            self.bycol = [np.flatnonzero(self.pcol == c) for c in range(self.npcol)]

    def _smooth(self, l, x, b, pre):
        if l != 0:
            return super()._smooth(l, x, b, pre)
        A0 = self.h.levels[0].A
        if self.l0kind == 'asm':
            return x + self.asm_w * (self.S @ (b - A0 @ x))
        for order in (range(self.npcol), range(self.npcol - 1, -1, -1)):
            for c in order:
                for k in self.bycol[c]:
                    p = self.pats[k]
                    x[p] += self.pinv[k] @ (b[p] - self.prow[k] @ x)
        return x


def run_patch(cases):
    for dim, n, g in cases:
        s = mo.bidomain_system(dim, n, g)
        A = s['A']
        b = mo.seeded_rhs(A.shape[0])
        out = dict(dim=dim, n=n, gamma=g)
        for name, kw in [('asm_V_bjac', dict(l0kind='asm')),
                         ('asm_V_mcsgs', dict(l0kind='asm', smoother='mcsgs')),
                         ('asm_W_mcsgs_s', dict(l0kind='asm', smoother='mcsgs', cycle='W', scaling=True)),
                         ('msm_V_mcsgs', dict(l0kind='msm', smoother='mcsgs'))]:
            st = PatchStudy(A, s['idofs'], **kw)
            out[name] = mo.pcg(A, st, b, 1e-8, 500).niters
            if kw['l0kind'] == 'asm':
                out[name + '_rho'] = round(st.rho, 3)
            else:
                out[name + '_ncol'] = st.npcol
        print(out, flush=True)
