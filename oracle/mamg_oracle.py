"""CPU restatement of the metric-AMG hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module.  The product (``metric-amg-examples_amd``)
never imports, links or calls it; it is the *checker*.

PARITY STATUS: **parity unpinned** against the reference.
The reference (anabudisa/metric-amg-examples) contains no solver code; the
hot path lives in HAZmath (C) behind cbc.block / haznics, none of which is in
``/root/reference`` or installable here.  There are no golden vectors,
recorded iteration counts or KATs in the reference.  This oracle therefore
restates a *precisely specified* algorithm profile ("mi355x_sa_v")
built from the reference's own call sites and parameter dictionaries, and is
itself pinned only by hand-checkable known-answer tests
(``tests/test_oracle.py``: 1-D Laplacian aggregation/RAP, P1 stencils, CG on
scipy's direct solve).

Reference anchors (file:line in /root/reference):
  * matrix definition        src/bidomain_2d.py:51-99  (a00/a01/a10/a11 :64-68,
                             Dirichlet tags (1,2) :73), 3-D reuse
                             src/bidomain_3d.py:119, BC faces src/utils.py:159-160,
                             177-178; defaults kappa1=2, kappa2=3
                             src/bidomain_3d.py:64-65
  * monolithic block order   src/bidomain_3d.py:124,138,154-155  ([u1; u2])
  * interface dofs           src/bidomain_3d.py:138 (all u2 dofs)
  * parameter keys           src/amg_parameters.py:67-89, src/utils.py:60-82
  * PCG call                 src/bidomain_3d.py:149-160 (tol 1e-8, maxiter 500,
                             niters = len(residuals)-1, cond from Lanczos)
  * [ext] cbc.block ``cgN``  preconditioned residual sqrt(<r,Br>), absolute
                             tolerance, eigenvalue estimates from the CG
                             alpha/beta tridiagonal (recalled; not in repo)

Floating-point contract (what makes the product's setup *bitwise* equal to
this oracle): every setup quantity is a fixed sequence of IEEE-754 binary64
operations -- no FMA contraction, sums accumulated sequentially in CSR order
starting from 0.0 (scipy's ``csr_matvec``/``csr_matmat`` order), exact zeros
produced by cancellation in a sparse product/difference dropped (scipy's
rule), row entries kept sorted by column.
"""
from __future__ import annotations

import dataclasses
import math
import numpy as np
import scipy.sparse as sp

# --------------------------------------------------------------------------
# deterministic hash (MIS-2 priorities); same uint32 arithmetic in C++/HIP
# --------------------------------------------------------------------------
_M32 = np.uint64(0xFFFFFFFF)


def hash32(i, level: int) -> np.ndarray:
    """lowbias-style integer hash of (index, level) -> uint32."""
    x = (np.asarray(i, dtype=np.uint64) & _M32)
    lv = np.uint64((int(level) * 0x85EBCA77) & 0xFFFFFFFF)
    x = (x * np.uint64(0x9E3779B1) + lv) & _M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & _M32
    x ^= x >> np.uint64(16)
    return x


# --------------------------------------------------------------------------
# problem generator: bidomain P1 on dolfin's structured meshes
# --------------------------------------------------------------------------
# Kuhn (path-simplex) split: every cell is a monotone lattice path from the
# cell's lower corner to its upper corner.  dolfin UnitSquareMesh(n,n) 'right'
# = paths (x,y),(y,x); UnitCubeMesh(n,n,n) = the 6 axis permutations.
_K_PATH = {2: np.array([[1, -1, 0], [-1, 2, -1], [0, -1, 1]], dtype=np.int64),
           3: np.array([[1, -1, 0, 0], [-1, 2, -1, 0], [0, -1, 2, -1],
                        [0, 0, -1, 1]], dtype=np.int64)}


def _paths(dim):
    import itertools
    return list(itertools.permutations(range(dim)))


def p1_integer_stencils(dim: int, n: int):
    """Integer-count stiffness (cK) and mass (cM) matrices on the vertex graph.

    K = kfac * cK with kfac = h/6 (3-D) or 1/2 (2-D); M = mfac * cM with
    mfac = h^3/120 (3-D) or h^2/24 (2-D).  Counts are exact integers, so the
    assembled values do not depend on assembly order.
    Returns (indptr, indices, cK, cM) CSR over nv=(n+1)^dim vertices, sorted.
    """
    nn = n + 1
    nv = nn ** dim
    stride = [1, nn, nn * nn][:dim]
    cells0 = np.arange(n ** dim, dtype=np.int64)
    # lower-corner vertex index of each cell
    coords = []
    rem = cells0.copy()
    for d in range(dim):
        coords.append(rem % n)
        rem //= n
    base = np.zeros_like(cells0)
    for d in range(dim):
        base += coords[d] * stride[d]
    Kloc = _K_PATH[dim]
    rows, cols, ck, cm = [], [], [], []
    for path in _paths(dim):
        verts = [base]
        cur = base
        for ax in path:
            cur = cur + stride[ax]
            verts.append(cur)
        for a in range(dim + 1):
            for b in range(dim + 1):
                rows.append(verts[a])
                cols.append(verts[b])
                ck.append(np.full(base.shape, Kloc[a, b], dtype=np.int64))
                cm.append(np.full(base.shape, 2 if a == b else 1, dtype=np.int64))
    key = np.concatenate(rows) * nv + np.concatenate(cols)
    uniq, inv = np.unique(key, return_inverse=True)       # sorted (row, col)
    cKv = np.bincount(inv, weights=np.concatenate(ck)).round().astype(np.int64)
    cMv = np.bincount(inv, weights=np.concatenate(cm)).round().astype(np.int64)
    r, c = uniq // nv, uniq % nv
    indptr = np.zeros(nv + 1, dtype=np.int64)
    np.add.at(indptr, r + 1, 1)
    indptr = np.cumsum(indptr)
    # pattern = mass pattern (every vertex pair sharing a cell; cM >= 1)
    return indptr, c.astype(np.int64), cKv, cMv


def bc_vertices(dim: int, n: int) -> np.ndarray:
    """Dirichlet vertices: x=0,1 in 2-D (tags 1,2, src/utils.py:159-160);
    z=0,1 in 3-D (tags 1,2, src/utils.py:177-178)."""
    nn = n + 1
    v = np.arange(nn ** dim, dtype=np.int64)
    if dim == 2:
        ax = v % nn                      # x coordinate index
    else:
        ax = v // (nn * nn)              # z coordinate index
    return (ax == 0) | (ax == n)


def bidomain_system(dim: int, n: int, gamma: float, kappa1: float = 2.0,
                    kappa2: float = 3.0):
    """Monolithic bidomain matrix [[k1 K + g M, -g M], [-g M, k2 K + g M]].

    Block order [u1; u2] as ii_convert produces (src/bidomain_3d.py:124,138).
    Dirichlet dofs (both fields) are eliminated symmetrically: row/column
    removed, diagonal 1.0.  Returns dict(A=csr, nv=, idofs=, bc=).
    """
    indptr, indices, cK, cM = p1_integer_stencils(dim, n)
    nv = len(indptr) - 1
    h = 1.0 / n
    if dim == 3:
        kf1 = kappa1 * h / 6.0
        kf2 = kappa2 * h / 6.0
        mf = gamma * h * h * h / 120.0
    else:
        kf1 = kappa1 / 2.0
        kf2 = kappa2 / 2.0
        mf = gamma * h * h / 24.0
    fK = cK.astype(np.float64)
    fM = cM.astype(np.float64)
    a11 = kf1 * fK + mf * fM
    a22 = kf2 * fK + mf * fM
    a12 = -(mf * fM)
    rlen = np.diff(indptr)
    r = np.repeat(np.arange(nv, dtype=np.int64), rlen)
    c = indices
    rows = np.concatenate([r, r, r + nv, r + nv])
    cols = np.concatenate([c, c + nv, c, c + nv])
    vals = np.concatenate([a11, a12, a12, a22])
    bcv = bc_vertices(dim, n)
    isbc = np.concatenate([bcv, bcv])
    keep = ~(isbc[rows] | isbc[cols])
    d = np.flatnonzero(isbc)
    rows = np.concatenate([rows[keep], d])
    cols = np.concatenate([cols[keep], d])
    vals = np.concatenate([vals[keep], np.ones(len(d))])
    N = 2 * nv
    A = _csr_from_coo_unique(rows, cols, vals, N, N)
    idofs = np.arange(nv, 2 * nv, dtype=np.int32)
    return dict(A=A, nv=nv, idofs=idofs, bc=isbc, dim=dim, n=n, gamma=gamma)


def _csr_from_coo_unique(rows, cols, vals, nr, nc):
    order = np.lexsort((cols, rows))
    rows, cols, vals = rows[order], cols[order], vals[order]
    indptr = np.zeros(nr + 1, dtype=np.int64)
    np.add.at(indptr, rows + 1, 1)
    indptr = np.cumsum(indptr)
    A = sp.csr_matrix((vals.astype(np.float64), cols.astype(np.int64), indptr),
                      shape=(nr, nc))
    A.has_sorted_indices = True
    return A


def laplace1d(n: int) -> sp.csr_matrix:
    """Tridiagonal [-1 2 -1] (KAT input)."""
    A = sp.diags([-np.ones(n - 1), 2 * np.ones(n), -np.ones(n - 1)], [-1, 0, 1],
                 format='csr')
    A.sort_indices()
    return A


# --------------------------------------------------------------------------
# setup
# --------------------------------------------------------------------------
@dataclasses.dataclass
class Params:
    """Algorithm profile; keys mirror src/amg_parameters.py:67-89 names."""
    AMG_type: str = 'SA'          # 'SA' | 'UA'
    cycle_type: str = 'V'         # 'V' | 'W'
    aggregation_type: str = 'MIS'  # 'MIS' (MIS-2) | 'HEM' (parallel heavy-edge matching, 2 passes) | 'VMB'
    max_levels: int = 20
    maxit: int = 1
    smoother: str = 'JACOBI_RHO'  # 'L1DIAG' | 'JACOBI' | 'JACOBI_RHO' | 'POLY' | 'GS' | 'SGS'
    relaxation: float = 4.0 / 3.0
    presmooth_iter: int = 1
    postsmooth_iter: int = 1
    coarse_dof: int = 100
    strong_coupled: float = 0.0   # SoC threshold theta
    Schwarz_levels: int = 1       # 1: seed-block Jacobi on level 0 (needs idofs)
    Schwarz_mmsize: int = 100     # max dofs per seed block
    Schwarz_maxlvl: int = 1       # 1: seed + joined 1-ring neighbours; 0: the seed's node (node blocks)
    Schwarz_type: int = 4         # 4 / 7: non-overlapping seed blocks (the level smoother); 5: additive overlapping rings;
                                  # 6: node patches (3 on the 1-rings of a nodal system resolves to 6)
    sa_omega: float = 4.0 / 3.0   # prolongator smoothing  w = sa_omega / rho
    rho_iters: int = 0            # 0: Gershgorin bound; >0: inf-norm power its
    max_coarse_dense: int = 8192
    num_functions: int = 1        # >1: nodal aggregation over field-major dofs
    node_block_smoother: int = 1  # nodal: node-block Jacobi where no seed blocks
    sa_block_diag: int = 1        # nodal: smooth P with node-block D^-1
    coarse_scaling: int = 0       # 1: e <- alpha e, alpha = <b_c, e> / <A_c e, e>
    poly_degree: int = 2          # POLY: Chebyshev degree (steps per smoothing)
    poly_ratio: float = 16.0      # POLY: interval [hi / poly_ratio, hi] of W A
    strength_measure: int = 1     # 1: theta relative to the row's largest coupling; 0: classical sqrt(a_ii a_jj)



def _rowsum_seq(A: sp.csr_matrix, x: np.ndarray) -> np.ndarray:
    """y_i = sum_j A_ij x_j accumulated sequentially in CSR order (csr_matvec)."""
    return A @ x


def _offdiag_row_max(n: int, r: np.ndarray, c: np.ndarray, v: np.ndarray) -> np.ndarray:
    """max over j != i of v_ij per row i (0 for rows without one)."""
    m = np.zeros(n)
    off = r != c
    np.maximum.at(m, r[off], v[off])
    return m


def strength(A: sp.csr_matrix, theta: float, measure: int = 1) -> sp.csr_matrix:
    """Symmetric SoC: j strong for i iff |a_ij| >= theta*max_{k != i}|a_ik|
    and |a_ij| > 1e-12*sqrt(|a_ii||a_jj|) (j != i); then S <- S | S^T.
    The threshold is relative to the row's largest coupling, so every row
    with a (numerically nonzero) coupling keeps a strong neighbour: measured
    against sqrt(|a_ii||a_jj|) instead, the mass-dominated coarse levels of
    the bidomain at gamma = 1e6 lost every connection at theta = 0.1 (the
    reference presets' strong_coupled, src/amg_parameters.py:57,79) and the
    hierarchy collapsed (3-D n = 128: 324-336 PCG iterations).
    measure 0 (STRENGTH_DIAG) is that classical rule, |a_ij| >=
    theta*sqrt(|a_ii||a_jj|) (Vanek, Mandel, Brezina 1996), kept selectable.
    Returns boolean-valued CSR (values 1.0), sorted, no diagonal."""
    n = A.shape[0]
    d = np.abs(A.diagonal())
    r = np.repeat(np.arange(n), np.diff(A.indptr))
    c = A.indices
    av = np.abs(A.data)
    s = np.sqrt(d[r] * d[c])
    m = _offdiag_row_max(n, r, c, av)
    ref = m[r] if measure == 1 else s
    strong = (r != c) & (av >= theta * ref) & (av > 1e-12 * s)
    S = sp.csr_matrix((np.ones(int(strong.sum())), (r[strong], c[strong])),
                      shape=(n, n))
    S = ((S + S.T) != 0).astype(np.float64).tocsr()
    S.sort_indices()
    return S


def _row_max(S: sp.csr_matrix, vals: np.ndarray) -> np.ndarray:
    """max over row neighbours of vals (uint64); 0 for empty rows."""
    n = S.shape[0]
    out = np.zeros(n, dtype=np.uint64)
    rl = np.diff(S.indptr)
    nz = np.flatnonzero(rl > 0)
    if len(nz):
        out[nz] = np.maximum.reduceat(vals[S.indices], S.indptr[nz])
    return out


ST_OUT, ST_UND, ST_IN = 0, 1, 2


def mis2(S: sp.csr_matrix, level: int) -> np.ndarray:
    """Distance-2 maximal independent set, round-synchronous, hash priorities.

    key_i = state<<62 | (prio & 0x7fffffff)<<31 | i.  Per round:
    m1 = max(key, rowmax(key)); m2 = max(m1, rowmax(m1)); undecided i with
    m2_i == key_i -> IN, with state(m2_i) == IN -> OUT.  Nodes with no strong
    neighbours start OUT (excluded from aggregation).
    Returns state array (uint8)."""
    n = S.shape[0]
    rl = np.diff(S.indptr)
    state = np.where(rl > 0, ST_UND, ST_OUT).astype(np.uint64)
    idx = np.arange(n, dtype=np.uint64)
    pr = hash32(np.arange(n), level) & np.uint64(0x7FFFFFFF)
    low = (pr << np.uint64(31)) | idx
    rounds = 0
    while True:
        und = state == ST_UND
        if not und.any():
            break
        key = (state << np.uint64(62)) | low
        m1 = np.maximum(key, _row_max(S, key))
        m2 = np.maximum(m1, _row_max(S, m1))
        win = und & (m2 == key)
        lose = und & ~win & ((m2 >> np.uint64(62)) == ST_IN)
        state = np.where(win, ST_IN, np.where(lose, ST_OUT, state))
        rounds += 1
        if rounds > 10000:
            raise RuntimeError('mis2 did not converge')
    return state.astype(np.uint8)


def node_strength(A: sp.csr_matrix, nf: int, theta: float, measure: int = 1):
    """Nodal strength for nf fields laid out field-major (dof = f*nv + I).

    s_IJ = sqrt(sum over the nf x nf block (I,J) of a^2), accumulated
    sequentially in CSR order (rows f*nv+I for f = 0..nf-1, columns sorted).
    J strong for I iff s_IJ >= theta*max_{K != I} s_IK and
    s_IJ > 1e-12*sqrt(s_II s_JJ) (J != I); then S <- S | S^T (see strength).
    Returns (S, Wn): strong pattern (values 1.0) and the s_IJ matrix."""
    n = A.shape[0]
    nv = n // nf
    r = np.repeat(np.arange(n), np.diff(A.indptr))
    I = r % nv
    J = A.indices % nv
    key = I * nv + J
    uniq, inv = np.unique(key, return_inverse=True)
    s2 = np.bincount(inv, weights=A.data * A.data)   # sequential, CSR order
    s = np.sqrt(s2)
    ui, uj = uniq // nv, uniq % nv
    Wn = _csr_from_coo_unique(ui, uj, s, nv, nv)
    d = np.zeros(nv)
    dmask = ui == uj
    d[ui[dmask]] = s[dmask]
    sd = np.sqrt(d[ui] * d[uj])
    m = _offdiag_row_max(nv, ui, uj, s)
    ref = m[ui] if measure == 1 else sd
    strong = (ui != uj) & (s >= theta * ref) & (s > 1e-12 * sd)
    S = sp.csr_matrix((np.ones(int(strong.sum())), (ui[strong], uj[strong])), shape=(nv, nv))
    S = ((S + S.T) != 0).astype(np.float64).tocsr()
    S.sort_indices()
    return S, Wn


def tentative_nodal(agg: np.ndarray, nagg: int, nf: int) -> sp.csr_matrix:
    """dof f*nv + I -> coarse dof f*nagg + agg[I] (one column per field and
    aggregate: the constant near-kernel of every field; coarse level stays
    field-major with nv_c = nagg)."""
    nv = len(agg)
    has = np.tile(agg >= 0, nf)
    cols = np.concatenate([f * nagg + agg for f in range(nf)])
    indptr = np.concatenate([[0], np.cumsum(has)]).astype(np.int64)
    T = sp.csr_matrix((np.ones(int(has.sum())), cols[has].astype(np.int64), indptr),
                      shape=(nf * nv, nf * nagg))
    T.has_sorted_indices = True
    return T


def node_blocks(n: int, nf: int):
    """block id per dof for nf x nf node blocks: bid(f*nv + I) = I."""
    nv = n // nf
    return np.tile(np.arange(nv, dtype=np.int64), nf), nv


def aggregate_mis2(Wabs: sp.csr_matrix, S: sp.csr_matrix, level: int):
    """MIS-2 aggregation.  Roots numbered in index order; distance-1
    neighbours join their (unique) adjacent root; remaining non-isolated nodes
    join the phase-2 aggregate of the strong neighbour with the largest
    weight (|a_ij|, or s_IJ for nodal aggregation; ties: smallest aggregate
    id).  Isolated nodes: agg = -1."""
    A = Wabs
    n = A.shape[0]
    state = mis2(S, level)
    roots = np.flatnonzero(state == ST_IN)
    agg = np.full(n, -1, dtype=np.int64)
    agg[roots] = np.arange(len(roots))
    # phase 2: neighbours of roots
    r = np.repeat(np.arange(n), np.diff(S.indptr))
    c = S.indices
    isroot = np.zeros(n, dtype=bool)
    isroot[roots] = True
    m = isroot[c] & ~isroot[r]
    agg2 = agg.copy()
    agg2[r[m]] = agg[c[m]]
    # phase 3: remaining non-isolated
    nonisol = np.diff(S.indptr) > 0
    need = nonisol & (agg2 < 0)
    if need.any():
        W = A.multiply(S).tocsr()        # weights on strong pattern
        W.sort_indices()
        wr = np.repeat(np.arange(n), np.diff(W.indptr))
        wc = W.indices
        wv = W.data
        cand = need[wr] & (agg2[wc] >= 0)
        cr, cw, ca = wr[cand], wv[cand], agg2[wc[cand]]
        order = np.lexsort((ca, -cw, cr))
        cr, ca = cr[order], ca[order]
        first = np.ones(len(cr), dtype=bool)
        first[1:] = cr[1:] != cr[:-1]
        agg3 = agg2.copy()
        agg3[cr[first]] = ca[first]
        # nodes adjacent (strongly) only through pattern entries absent from A
        if (nonisol & (agg3 < 0)).any():
            raise RuntimeError('aggregation left a non-isolated node unassigned')
        agg2 = agg3
    return agg2, len(roots)


# --------------------------------------------------------------------------
# parallel heavy-edge matching aggregation (aggregation_type HEM,
# src/amg_parameters.py:79): HAZmath matches greedily in index order; here
# every pass is a round-synchronous handshake (locally dominant edges), so
# the GPU reproduces it exactly.  Two passes -> aggregates of <= 4 nodes.
# --------------------------------------------------------------------------
HEM_PASSES = 2
HEM_MAX_ROUNDS = 64


def edge_hash(i: np.ndarray, j: np.ndarray, level: int) -> np.ndarray:
    """symmetric 32-bit edge priority: hash32(min) ^ hash32(max) (host.h hash32)"""
    a, b = np.minimum(i, j), np.maximum(i, j)
    return hash32(a, 0x5000 + level) ^ hash32(b, 0x6000 + level)


def hem_match(W: sp.csr_matrix, active: np.ndarray, level: int):
    """Handshake matching on the weighted graph W (symmetric, no diagonal):
    per round every free active node picks the free neighbour with the
    largest (weight, edge hash, -index); mutual picks are matched.  Rounds
    until none is matched (at most HEM_MAX_ROUNDS).  Returns mate (-1 free)."""
    n = W.shape[0]
    r = np.repeat(np.arange(n), np.diff(W.indptr))
    c = W.indices.astype(np.int64)
    w = W.data
    h = edge_hash(r, c, level).astype(np.int64)
    mate = np.full(n, -1, dtype=np.int64)
    for _ in range(HEM_MAX_ROUNDS):
        free = active & (mate < 0)
        m = free[r] & free[c] & (r != c)
        rr, cc, ww, hh = r[m], c[m], w[m], h[m]
        order = np.lexsort((cc, -hh, -ww, rr))          # row asc; weight, hash desc; col asc
        rr, cc = rr[order], cc[order]
        first = np.ones(len(rr), dtype=bool)
        first[1:] = rr[1:] != rr[:-1]
        choice = np.full(n, -1, dtype=np.int64)
        choice[rr[first]] = cc[first]
        i = np.flatnonzero(choice >= 0)
        mutual = i[choice[choice[i]] == i]
        if len(mutual) == 0:
            break
        mate[mutual] = choice[mutual]
    return mate


def aggregate_vmb(Wabs: sp.csr_matrix, S: sp.csr_matrix, level: int):
    """Vanek-Mandel-Brezina aggregation (aggregation_type VMB, the
    reference's parameters_standard, src/amg_parameters.py:16,36, and the
    3D-1D .dat file, src/input_metric.dat:89), sequential, in index order.
    HAZmath's own VMB source is absent, so this is the
    published algorithm (Vanek, Mandel, Brezina 1996, section 3):
      phase 1: node i, non-isolated, with itself and every strong neighbour
               still free -> a new aggregate {i} + N(i);
      phase 2: every remaining non-isolated node joins the phase-1 aggregate
               of its strong neighbour with the largest weight (|a_ij|, or
               s_IJ for nodal aggregation; ties: smallest aggregate id).
    Every non-isolated node left free by phase 1 has a phase-1-aggregated
    strong neighbour (else phase 1 would have started an aggregate at it).
    Isolated nodes: agg = -1.  `level` is unused (no random priorities)."""
    n = S.shape[0]
    ip, ix = S.indptr, S.indices
    agg = np.full(n, -1, dtype=np.int64)
    nagg = 0
    for i in range(n):
        if ip[i + 1] == ip[i] or agg[i] >= 0:
            continue
        nb = ix[ip[i]:ip[i + 1]]
        if (agg[nb] >= 0).any():
            continue
        agg[i] = nagg
        agg[nb] = nagg
        nagg += 1
    agg1 = agg.copy()
    need = (np.diff(ip) > 0) & (agg1 < 0)
    if need.any():
        W = Wabs.multiply(S).tocsr()
        W.sort_indices()
        for i in np.flatnonzero(need):
            cols = W.indices[W.indptr[i]:W.indptr[i + 1]]
            ws = W.data[W.indptr[i]:W.indptr[i + 1]]
            best_w, best_a = -1.0, -1
            for j, w in zip(cols, ws):
                a = agg1[j]
                if w == 0.0 or a < 0:
                    continue
                if w > best_w or (w == best_w and a < best_a):
                    best_w, best_a = w, a
            if best_a < 0:
                raise RuntimeError('aggregation left a non-isolated node unassigned')
            agg[i] = best_a
    return agg, nagg


def aggregate_hem(Wabs: sp.csr_matrix, S: sp.csr_matrix, level: int):
    """HEM_PASSES handshake passes on the strong graph weighted by |a_ij| /
    s_IJ; pass k+1 matches the aggregates of pass k on W_k+1 = T_k^T W_k T_k
    (SMMP products, diagonal and zeros dropped).  Aggregates are numbered by
    their smallest member in index order; isolated nodes: -1."""
    n = Wabs.shape[0]
    W = Wabs.multiply(S).tocsr()
    W.eliminate_zeros()
    W.sort_indices()
    active = np.diff(S.indptr) > 0
    agg = np.where(active, np.arange(n), -1)
    cur, act = W, active
    nagg = n
    if not active.any():             # no strong edge (e.g. theta > 0 on a coarse level): no aggregates
        return np.full(n, -1, dtype=np.int64), 0
    for ps in range(HEM_PASSES):
        m = cur.shape[0]
        mate = hem_match(cur, act, 16 * level + ps)
        idx = np.arange(m)
        root = np.where(mate >= 0, np.minimum(idx, mate), idx)
        isroot = act & (root == idx)
        num = np.cumsum(isroot) - 1
        a = np.where(act, num[root], -1)
        nagg = int(isroot.sum())
        agg = np.where(agg >= 0, a[np.maximum(agg, 0)], -1)
        if ps + 1 == HEM_PASSES:
            break
        rows = np.flatnonzero(act)
        T = sp.csr_matrix((np.ones(len(rows)), (rows, a[rows])), shape=(m, nagg))
        T.sort_indices()
        WT = (cur @ T).tocsr()
        WT.sort_indices()
        C = (T.T.tocsr() @ WT).tocsr()
        C.sort_indices()
        C.setdiag(0.0)
        C.eliminate_zeros()
        C.sort_indices()
        cur = C
        act = np.ones(nagg, dtype=bool)   # every aggregate may match (no external edge: stays alone)
    # a node left alone by every pass joins the aggregate of its heaviest
    # strong neighbour that has >= 2 members (ties: smallest aggregate id);
    # the aggregates are then renumbered in order (matching alone leaves the
    # leaves of star-like coarse graphs unmatched and coarsening stalls)
    size = np.bincount(agg[agg >= 0], minlength=nagg)
    r = np.repeat(np.arange(n), np.diff(W.indptr))
    c = W.indices
    single = (agg >= 0) & (size[np.maximum(agg, 0)] == 1)
    m = single[r] & (agg[c] >= 0) & (size[np.maximum(agg[c], 0)] >= 2)
    rr, ww, aa = r[m], W.data[m], agg[c[m]]
    order = np.lexsort((aa, -ww, rr))
    rr, aa = rr[order], aa[order]
    first = np.ones(len(rr), dtype=bool)
    first[1:] = rr[1:] != rr[:-1]
    agg2 = agg.copy()
    agg2[rr[first]] = aa[first]
    used = np.zeros(nagg, dtype=bool)
    used[agg2[agg2 >= 0]] = True
    newid = np.cumsum(used) - 1
    agg2 = np.where(agg2 >= 0, newid[np.maximum(agg2, 0)], -1)
    return agg2, int(used.sum())


def tentative(agg: np.ndarray, nagg: int) -> sp.csr_matrix:
    n = len(agg)
    has = agg >= 0
    indptr = np.concatenate([[0], np.cumsum(has)]).astype(np.int64)
    T = sp.csr_matrix((np.ones(int(has.sum())), agg[has].astype(np.int64), indptr),
                      shape=(n, nagg))
    T.has_sorted_indices = True
    return T


def rho_estimate(A: sp.csr_matrix, dinv: np.ndarray, iters: int) -> float:
    """Estimate rho(D^-1 A).  iters == 0: Gershgorin bound
    max_i dinv_i * sum_j |a_ij|.  iters > 0: inf-norm power iteration from a
    hash-based start vector."""
    absA = abs(A)
    if iters == 0:
        rs = _rowsum_seq(absA, np.ones(A.shape[0]))
        return float(np.max(dinv * rs))
    n = A.shape[0]
    v = (hash32(np.arange(n), 977).astype(np.float64) / 4294967296.0) * 2.0 - 1.0
    rho = 0.0
    for _ in range(iters):
        w = dinv * _rowsum_seq(A, v)
        mv = float(np.max(np.abs(v)))
        mw = float(np.max(np.abs(w)))
        rho = mw / mv
        v = w / mw
    return rho


def smooth_prolongator(A, T, omega_sa, rho_iters):
    """P = T - (w * dinv) (A T), w = omega_sa / rho(D^-1 A), dinv = 1/a_ii."""
    dinv = 1.0 / A.diagonal()
    rho = rho_estimate(A, dinv, rho_iters)
    w = omega_sa / rho
    AT = (A @ T).tocsr()
    AT.sort_indices()
    c = w * dinv
    X = (sp.diags(c, format='csr') @ AT).tocsr()
    P = (T - X).tocsr()
    P.sort_indices()
    return P, w


def smooth_prolongator_block(A, T, omega_sa, blocks):
    """Nodal SA: P = T - w (D_B^-1 (A T)), D_B = node-block diagonal,
    w = omega_sa / rho_B, rho_B = max_i sum_j |(D_B^-1 A)_ij|."""
    bid, nb = blocks
    Dinv = block_inverse_csr(A, bid, nb)
    G = (Dinv @ A).tocsr()
    G.sort_indices()
    rho = float(np.max(_rowsum_seq(abs(G), np.ones(A.shape[0]))))
    w = omega_sa / rho
    AT = (A @ T).tocsr()
    AT.sort_indices()
    Y = (Dinv @ AT).tocsr()
    Y.sort_indices()
    Y.data = w * Y.data
    P = (T - Y).tocsr()
    P.sort_indices()
    return P, w


def galerkin(A, P):
    """R = P^T (sorted CSR); A_c = R @ (A @ P), both products in SMMP order."""
    R = P.T.tocsr()
    R.sort_indices()
    AP = (A @ P).tocsr()
    AP.sort_indices()
    Ac = (R @ AP).tocsr()
    Ac.sort_indices()
    return R, Ac


def smoother_weights(A, p: Params):
    """winv_i = relaxation / d_i with d_i = a_ii (JACOBI) or sum_j |a_ij|
    (L1DIAG, sequential CSR-order sum); JACOBI_RHO: d_i = a_ii * rho(D^-1 A)
    (spectrally scaled Jacobi, same rho estimate as prolongator smoothing)."""
    if p.smoother == 'JACOBI':
        d = A.diagonal().copy()
    elif p.smoother in ('JACOBI_RHO', 'POLY'):
        dg = A.diagonal().copy()
        rho = rho_estimate(A, 1.0 / dg, p.rho_iters)
        d = dg * rho
    elif p.smoother == 'L1DIAG':
        d = _rowsum_seq(abs(A), np.ones(A.shape[0]))
    else:
        raise ValueError(p.smoother)
    return p.relaxation / d


def poly_weights(p: Params) -> list:
    """POLY smoother step weights (product form of the Chebyshev polynomial).

    The block smoother W = (relaxation / rho_B) D^-1 bounds the spectrum of
    W A by hi = relaxation (rho_B is a Gershgorin bound of rho(D^-1 A)).  The
    degree-m Chebyshev polynomial on [hi / poly_ratio, hi] is the product of
    m Richardson steps x += w_k W (b - A x) with w_k = 1 / tau_k, tau_k its
    roots theta + delta cos((2k - 1) pi / (2m)), k = 1..m (ascending k =
    descending tau).  Pre-smoothing takes the steps in order 1..m,
    post-smoothing m..1, so the cycle stays symmetric.  Same formula as
    device.hip poly_weights (C, libm cos)."""
    m = int(p.poly_degree)
    hi = float(p.relaxation)
    lo = hi / float(p.poly_ratio)
    theta, delta = 0.5 * (hi + lo), 0.5 * (hi - lo)
    return [1.0 / (theta + delta * math.cos((2 * k - 1) * math.pi / (2 * m))) for k in range(1, m + 1)]


def scaled_smoother(lev, w: float):
    """w * W of a level (block CSR or point weights), scaled value by value."""
    if lev.WB is not None:
        W = lev.WB.copy()
        W.data = w * W.data
        return W
    return w * lev.winv


def dense_inverse(Ad: np.ndarray) -> np.ndarray:
    """Gauss-Jordan without pivoting (A SPD); fixed op order:
    row_k /= p;  row_i -= M_ik * row_k  (product, then subtraction)."""
    return batched_inverse(Ad[None, :, :])[0]


def batched_inverse(B: np.ndarray) -> np.ndarray:
    """Gauss-Jordan (no pivoting) on a batch (nb, s, s); same op order as
    ``dense_inverse`` applied block by block."""
    nb, n, _ = B.shape
    M = np.concatenate([B.astype(np.float64),
                        np.broadcast_to(np.eye(n), (nb, n, n))], axis=2).copy()
    for k in range(n):
        p = M[:, k, k].copy()
        if not np.all(p > 0.0):
            raise np.linalg.LinAlgError('non-positive pivot at %d' % k)
        M[:, k, :] = M[:, k, :] / p[:, None]
        f = M[:, :, k].copy()
        f[:, k] = 0.0
        M -= f[:, :, None] * M[:, k, None, :]
    return M[:, :, n:].copy()


def seed_blocks(A: sp.csr_matrix, seeds: np.ndarray, mmsize: int):
    """Non-overlapping Schwarz blocks seeded by ``idofs`` (src/utils.py:84-86).

    Each non-seed dof j joins the block of the seed s maximising |a_js| over
    j's off-diagonal seed neighbours (ties: smallest s); a seed's block keeps
    at most mmsize-1 joiners (lowest indices), the rest stay singletons.
    Blocks are numbered by their owner (seed or singleton) index; dofs inside
    a block are sorted.  Returns (bid[n], nblocks)."""
    n = A.shape[0]
    isseed = np.zeros(n, dtype=bool)
    isseed[np.asarray(seeds, dtype=np.int64)] = True
    r = np.repeat(np.arange(n), np.diff(A.indptr))
    c = A.indices
    v = np.abs(A.data)
    m = (~isseed[r]) & isseed[c] & (r != c)
    cr, cc, cv = r[m], c[m], v[m]
    order = np.lexsort((cc, -cv, cr))
    cr, cc = cr[order], cc[order]
    first = np.ones(len(cr), dtype=bool)
    first[1:] = cr[1:] != cr[:-1]
    jr, js = cr[first], cc[first]            # joiner -> seed (jr ascending)
    # cap joiners per seed at mmsize-1 (lowest joiner indices kept)
    o2 = np.lexsort((jr, js))
    jr, js = jr[o2], js[o2]
    newgrp = np.ones(len(js), dtype=bool)
    newgrp[1:] = js[1:] != js[:-1]
    grpstart = np.maximum.accumulate(np.where(newgrp, np.arange(len(js)), 0))
    rank = np.arange(len(js)) - grpstart
    keep = rank < (mmsize - 1)
    owner = np.arange(n)
    owner[jr[keep]] = js[keep]
    uo, bid = np.unique(owner, return_inverse=True)
    return bid.astype(np.int64), len(uo)


def block_inverse_csr(A: sp.csr_matrix, bid: np.ndarray, nb: int):
    """D_B^-1 as CSR: row i holds (D_B^-1)_{ij} for j in block(i), sorted."""
    n = A.shape[0]
    order = np.lexsort((np.arange(n), bid))          # dofs grouped by block
    starts = np.searchsorted(bid[order], np.arange(nb + 1))
    size = np.diff(starts)
    pos = np.empty(n, dtype=np.int64)
    pos[order] = np.arange(n) - np.repeat(starts[:-1], size)
    r = np.repeat(np.arange(n), np.diff(A.indptr))
    c = A.indices
    inb = bid[r] == bid[c]
    rows_out, cols_out, vals_out = [], [], []
    for s in np.unique(size):
        blks = np.flatnonzero(size == s)
        loc = np.full(nb, -1, dtype=np.int64)
        loc[blks] = np.arange(len(blks))
        dense = np.zeros((len(blks), s, s))
        m = inb & (size[bid[r]] == s)
        dense[loc[bid[r[m]]], pos[r[m]], pos[c[m]]] = A.data[m]
        inv = batched_inverse(dense)
        members = order[np.repeat(starts[blks], s) + np.tile(np.arange(s), len(blks))]
        members = members.reshape(len(blks), s)
        rr = np.repeat(members, s, axis=1).ravel()        # row dof
        cc = np.tile(members, (1, s)).ravel()             # col dof
        rows_out.append(rr)
        cols_out.append(cc)
        vals_out.append(inv.reshape(len(blks), s * s))
    rows = np.concatenate(rows_out)
    cols = np.concatenate(cols_out)
    vals = np.concatenate([v.ravel() for v in vals_out])
    return _csr_from_coo_unique(rows, cols, vals, n, n)


def block_smoother(A: sp.csr_matrix, seeds, p: Params, blocks=None) -> sp.csr_matrix:
    """W_B = (relaxation / rho_B) D_B^-1, rho_B = max_i sum_j |(D_B^-1 A)_ij|
    (Gershgorin bound; SpGEMM in SMMP order, sequential abs row sums).
    Blocks: seed blocks from ``seeds``, or an explicit (bid, nb)."""
    if blocks is None:
        bid, nb = seed_blocks(A, seeds, p.Schwarz_mmsize)
    else:
        bid, nb = blocks
    Dinv = block_inverse_csr(A, bid, nb)
    G = (Dinv @ A).tocsr()
    G.sort_indices()
    rho = float(np.max(_rowsum_seq(abs(G), np.ones(A.shape[0]))))
    s = p.relaxation / rho
    W = Dinv.copy()
    W.data = s * W.data
    return W, bid, nb


# --------------------------------------------------------------------------
# additive overlapping Schwarz on the seeds' rings (Schwarz_type ADDITIVE):
# the reference's seed + Schwarz_maxlvl-ring blocks (src/amg_parameters.py:
# 83-86, src/input_metric.dat:96-100) smoothed additively, so the blocks can
# overlap and every block works in parallel; dofs in no block take 1/a_ii
# --------------------------------------------------------------------------
SCHWARZ_ADDITIVE = 5


def seed_ring_blocks(A: sp.csr_matrix, seeds, maxlvl: int, mmsize: int):
    """Per seed (in the given order): the seed, then breadth-first its graph
    neighbours up to distance maxlvl, each vertex's neighbours in ascending
    order, stopping at mmsize dofs; members sorted."""
    ip, ix = A.indptr, A.indices
    blocks = []
    for s0 in np.asarray(seeds, dtype=np.int64):
        s0 = int(s0)
        seen = {s0}
        order = [s0]
        head = 0
        depth = {s0: 0}
        while head < len(order) and len(order) < mmsize:
            v = order[head]
            head += 1
            if depth[v] == maxlvl:
                continue
            for j in ix[ip[v]:ip[v + 1]]:
                j = int(j)
                if j not in seen:
                    seen.add(j)
                    order.append(j)
                    depth[j] = depth[v] + 1
                    if len(order) >= mmsize:
                        break
        blocks.append(np.array(sorted(order), dtype=np.int64))
    return blocks


def overlap_smoother(A: sp.csr_matrix, seeds, p: 'Params'):
    """W = (relaxation / lambda) S,  S = sum_k R_k^T A_k^-1 R_k (+ 1/a_ii on
    dofs in no block).  A_k^-1 by Gauss-Jordan; S accumulated block by block
    (k ascending, rows then columns of each block) on its sorted pattern from
    0.0; lambda = max(rho_iters, 30) inf-norm power iterations of S A from
    the hash start vector (the spectrum of an overlapping sum is far below
    its Gershgorin bound).  Returns (W, blocks)."""
    A = A.tocsr()
    n = A.shape[0]
    blocks = seed_ring_blocks(A, seeds, p.Schwarz_maxlvl, p.Schwarz_mmsize)
    cov = np.zeros(n, dtype=bool)
    rows, cols = [], []
    for b in blocks:
        cov[b] = True
        rows.append(np.repeat(b, len(b)))
        cols.append(np.tile(b, len(b)))
    unc = np.flatnonzero(~cov)
    rows.append(unc)
    cols.append(unc)
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    key = np.unique(r * n + c)
    pr, pc = key // n, key % n
    indptr = np.concatenate([[0], np.cumsum(np.bincount(pr, minlength=n))]).astype(np.int64)
    data = np.zeros(len(key))
    for b in blocks:
        dense = A[b][:, b].toarray()
        Ki = batched_inverse(dense[None, :, :])[0]
        pos = np.searchsorted(key, (np.repeat(b, len(b)) * n + np.tile(b, len(b))))
        for t in range(len(pos)):          # sequential: duplicates in block order
            data[pos[t]] += Ki.ravel()[t]
    if len(unc):
        pos = np.searchsorted(key, unc * n + unc)
        data[pos] = 1.0 / A.diagonal()[unc]
    S = sp.csr_matrix((data, pc.astype(np.int64), indptr), shape=(n, n))
    S.has_sorted_indices = True
    v = (hash32(np.arange(n), 977).astype(np.float64) / 4294967296.0) * 2.0 - 1.0
    lam = 0.0
    for _ in range(max(int(p.rho_iters), 30)):
        w = _rowsum_seq(S, _rowsum_seq(A, v))
        mv, mw = float(np.max(np.abs(v))), float(np.max(np.abs(w)))
        lam = mw / mv
        v = w / mw
    W = S.copy()
    W.data = (p.relaxation / lam) * W.data
    return W, blocks


# --------------------------------------------------------------------------
# multicolour node-block Gauss-Seidel (the reference's SGS smoother,
# src/amg_parameters.py:72, and its level-0 multiplicative Schwarz on the seed
# blocks, src/utils.py:84 / amg_parameters.py:83-86, in a GPU-parallel order)
# --------------------------------------------------------------------------
GS_MAX_COLOURS = 64


def node_pattern(A: sp.csr_matrix, nf: int) -> sp.csr_matrix:
    """Node graph of a field-major dof matrix: block (I, J) present iff any
    entry of rows f*nv+I lies in columns g*nv+J; diagonal excluded.  Raises if
    the pattern is not symmetric (the colouring needs an undirected graph)."""
    n = A.shape[0]
    nv = n // nf
    r = np.repeat(np.arange(n), np.diff(A.indptr)) % nv
    c = A.indices % nv
    m = r != c
    G = sp.csr_matrix((np.ones(int(m.sum()), np.int8), (r[m], c[m])), shape=(nv, nv))
    G.sum_duplicates()
    G.data[:] = 1
    G.sort_indices()
    if (G != G.T).nnz:
        raise RuntimeError('node pattern not symmetric: multicolour GS unsupported')
    return G


def colour_key(nv: int, level: int) -> np.ndarray:
    """priority of node I: hash32(I, level + 0x4000) in the high word, I in
    the low word (unique)."""
    I = np.arange(nv, dtype=np.uint64)
    return (hash32(np.arange(nv), level + 0x4000).astype(np.uint64) << np.uint64(32)) | I


def jp_colouring(G: sp.csr_matrix, level: int) -> np.ndarray:
    """Round-synchronous Jones-Plassmann colouring.  Per round every
    uncoloured node whose key exceeds the keys of all its uncoloured
    neighbours takes the smallest colour held by none of its (previously)
    coloured neighbours.  Winners of one round are never adjacent, so the
    result does not depend on the order nodes are visited (the GPU kernel
    runs the same rounds).  Returns int32 colour per node."""
    nv = G.shape[0]
    key = colour_key(nv, level)
    col = np.full(nv, -1, np.int64)
    ip, ix = G.indptr, G.indices
    rr = np.repeat(np.arange(nv), np.diff(ip))
    rounds = 0
    while (col < 0).any():
        unc = col < 0
        kk = np.where(unc, key, np.uint64(0))
        nbmax = np.zeros(nv, np.uint64)
        if len(ix):
            nz = np.flatnonzero(np.diff(ip) > 0)
            nbmax[nz] = np.maximum.reduceat(kk[ix], ip[nz])
        win = unc & (key > nbmax)
        bits = np.where(col[ix] >= 0, np.left_shift(np.uint64(1), np.maximum(col[ix], 0).astype(np.uint64)),
                        np.uint64(0))
        mask = np.zeros(nv, np.uint64)
        if len(ix):
            mask[nz] = np.bitwise_or.reduceat(bits, ip[nz])
        w = np.flatnonzero(win)
        m = mask[w]
        if np.any(m == np.uint64(0xFFFFFFFFFFFFFFFF)):
            raise RuntimeError('more than %d colours' % GS_MAX_COLOURS)
        free = (~m) & (m + np.uint64(1))            # lowest zero bit
        c = np.zeros(len(w), np.int64)
        for b in range(GS_MAX_COLOURS):
            c[free == (np.uint64(1) << np.uint64(b))] = b
        col[w] = c
        rounds += 1
    return col.astype(np.int32)


def node_block_inverse(A: sp.csr_matrix, bid: np.ndarray, nb: int, nf: int = 2) -> np.ndarray:
    """Unscaled inverse of the smoother blocks as one nf x nf block per node
    (nv, nf, nf); blocks must be node-aligned (both dofs of a node in one
    block, or each alone).  Same Gauss-Jordan as block_inverse_csr."""
    n = A.shape[0]
    nv = n // nf
    Dinv = block_inverse_csr(A, bid, nb)
    out = np.zeros((nv, nf, nf))
    for f in range(nf):
        for g in range(nf):
            rows = f * nv + np.arange(nv)
            cols = g * nv + np.arange(nv)
            out[:, f, g] = np.asarray(Dinv[rows, cols]).ravel()
    same = np.all([bid[f * nv:(f + 1) * nv] == bid[:nv] for f in range(nf)], axis=0)
    sizes = np.bincount(bid, minlength=nb)
    if not np.all(same | (sizes[bid[:nv]] == 1)):
        raise RuntimeError('smoother blocks not node-aligned: multicolour GS unsupported')
    return out


# --------------------------------------------------------------------------
# Multiplicative node-patch Schwarz on level 0 (Schwarz_type PATCHES): the
# reference's level-0 smoother -- symmetric multiplicative Schwarz on one
# block per seed = the seed + its Schwarz_maxlvl = 1 ring in A's graph
# (src/amg_parameters.py:83-87, src/utils.py:84), exact local solves
# (Schwarz_blksolver 32).  With the bidomain's seeds (every u2 dof,
# src/bidomain_3d.py:138) the block of node I's seed is both fields of the
# closed node neighbourhood N[I].  Parallel order: patches coloured so that
# two patches of one colour are >= 4 node hops apart (distance-3
# Jones-Plassmann), so no patch of a colour reads an x another one writes;
# a sweep takes the colours in order (forward) or reversed (backward).
# --------------------------------------------------------------------------
SCHWARZ_PATCHES = 6
PATCH_MAX_NODES = 16
PATCH_MAX_COLOURS = 256


def patch_key(nv: int) -> np.ndarray:
    """priority of patch (centre node) I: hash32(I, 0x5000) high, I low."""
    I = np.arange(nv, dtype=np.uint64)
    return (hash32(np.arange(nv), 0x5000).astype(np.uint64) << np.uint64(32)) | I


def _row_reduce(Gd: sp.csr_matrix, v: np.ndarray, op) -> np.ndarray:
    """out[I] = op over the columns J of row I of v[J] (rows are non-empty)."""
    return op.reduceat(v[Gd.indices], Gd.indptr[:-1], axis=0)


def patch_colouring(Gd: sp.csr_matrix) -> np.ndarray:
    """Distance-3 round-synchronous Jones-Plassmann on the node graph Gd
    (diagonal included).  Per round: k3 = max over the 3-hop neighbourhood
    of the uncoloured keys (three row-max passes), m3 = OR over the 3-hop
    neighbourhood of the coloured nodes' colour bits (256-bit, four uint64
    words); an uncoloured node with k3 == its own key takes the lowest colour
    absent from m3.  Two winners of a round are > 3 hops apart, so the
    result does not depend on the visiting order (device: patch_round)."""
    nv = Gd.shape[0]
    key = patch_key(nv)
    col = np.full(nv, -1, np.int64)
    words = PATCH_MAX_COLOURS // 64
    while (col < 0).any():
        unc = col < 0
        k = np.where(unc, key, np.uint64(0))
        for _ in range(3):
            k = _row_reduce(Gd, k, np.maximum)
        m = np.zeros((nv, words), np.uint64)
        cc = np.flatnonzero(~unc)
        m[cc, col[cc] // 64] = np.left_shift(np.uint64(1), (col[cc] % 64).astype(np.uint64))
        for _ in range(3):
            m = _row_reduce(Gd, m, np.bitwise_or)
        win = np.flatnonzero(unc & (k == key))
        c = np.full(len(win), -1, np.int64)
        for wd in range(words - 1, -1, -1):
            mw = m[win, wd]
            free = (~mw) & (mw + np.uint64(1))      # lowest zero bit of the word
            has = free != 0
            c[has] = 64 * wd + np.log2(free[has].astype(np.float64)).astype(np.int64)
        if (c < 0).any():
            raise RuntimeError('more than %d patch colours' % PATCH_MAX_COLOURS)
        col[win] = c
    return col.astype(np.int32)


class Patches:
    """Level-0 node patches: centre I -> nodes = row I of the node graph with
    its diagonal (sorted); local dof i = 2 a + f (a = position of the node,
    f = field); Minv = the patch matrix's Gauss-Jordan inverse (no pivoting,
    batched_inverse), symmetrised from its upper triangle."""

    def __init__(self, A: sp.csr_matrix, idofs):
        n = A.shape[0]
        nv = n // 2
        if idofs is None or np.unique(np.asarray(idofs, np.int64) % nv).size != nv:
            raise ValueError('node patches need a seed dof on every node')
        G = node_pattern(A, 2)
        Gd = (G + sp.identity(nv, dtype=np.int8, format='csr')).tocsr()
        Gd.data[:] = 1
        Gd.sort_indices()
        m = np.diff(Gd.indptr)
        if m.max() > PATCH_MAX_NODES:
            raise RuntimeError('a node patch holds more than %d nodes' % PATCH_MAX_NODES)
        self.nv = nv
        self.colour = patch_colouring(Gd)
        self.ncolours = int(self.colour.max()) + 1
        self.crows = [np.flatnonzero(self.colour == c) for c in range(self.ncolours)]
        self.m = m
        dmax = 2 * int(m.max())
        # dofs[I, i] = global dof of local dof i (field-major order), -1 padding
        self.dofs = np.full((nv, dmax), -1, np.int64)
        self.Minv = np.zeros((nv, dmax, dmax))
        A = A.tocsr()
        for mm in np.unique(m):
            I = np.flatnonzero(m == mm)
            nodes = np.stack([Gd.indices[Gd.indptr[i]:Gd.indptr[i + 1]] for i in I])   # (k, mm)
            d = 2 * mm
            dofs = np.empty((len(I), d), np.int64)
            dofs[:, 0::2] = nodes
            dofs[:, 1::2] = nv + nodes
            self.dofs[I, :d] = dofs
            Ap = np.stack([A[dd][:, dd].toarray() for dd in dofs])
            Mi = batched_inverse(Ap)
            U = np.triu(Mi)
            self.Minv[I, :d, :d] = U + np.transpose(np.triu(Mi, 1), (0, 2, 1))

    def sweep(self, A: sp.csr_matrix, x: np.ndarray, b: np.ndarray, forward=True):
        """x <- x + Minv_I (b - A x)|_patch(I) for the patches of each colour
        in turn (ascending if forward, else descending)."""
        order = range(self.ncolours) if forward else range(self.ncolours - 1, -1, -1)
        for c in order:
            I = self.crows[c]
            D = self.dofs[I]
            ok = D >= 0
            dd = D[ok]
            res = np.zeros(D.shape)
            res[ok] = b[dd] - A[dd] @ x
            delta = np.einsum('kij,kj->ki', self.Minv[I], res)
            x[dd] = x[dd] + delta[ok]
        return x


# --------------------------------------------------------------------------
# Multiplicative Schwarz on the seeds' overlapping rings (Schwarz_type RINGS):
# the reference's level-0 smoother for sparse seed sets.  The EMI drivers call
# get_hazmath_metric_precond without parameters (src/emi_3d.py:133-139), i.e.
# the default dict of src/utils.py:60-82: SCHWARZ_SYMMETRIC on seed +
# Schwarz_maxlvl = 2 ring blocks of at most Schwarz_mmsize = 100 dofs, seeded
# by the interface dofs of both sides; "the interface_dofs has the Schwarz and
# the rest the GS smoother" (src/utils.py:84).  Restated in a parallel order:
# * one block per seed, in the given seed order (seed_ring_blocks), exact
#   local solves (Gauss-Jordan, batched_inverse);
# * blocks k and l conflict iff a member of one lies in the closed
#   neighbourhood (A's pattern) of a member of the other; greedy first-fit
#   colouring in seed order, so no block of a colour writes an x another block
#   of that colour reads, and one colour is one parallel update;
# * the rest: node-block Gauss-Seidel restricted to the dofs in no block, in
#   the multicolour node order of the level-0 GS (jp_colouring): a node with
#   both dofs uncovered takes its 2x2 block inverse, a node with one its
#   1 / a_ii, a covered dof no update;
# * one symmetric step = ring sweep forward (colours ascending), rest GS
#   forward, rest GS backward, ring sweep backward -- palindromic, so the
#   same step serves pre- and post-smoothing and the cycle stays symmetric.
# --------------------------------------------------------------------------
SCHWARZ_RINGS = 8


def ring_colouring(A: sp.csr_matrix, blocks) -> np.ndarray:
    """Greedy first-fit colour of every ring block in block (= seed) order on
    the conflict graph (member of one block in the closed neighbourhood of a
    member of the other).  Returns int32 colour per block."""
    n = A.shape[0]
    nb = len(blocks)
    if nb == 0:
        return np.zeros(0, np.int32)
    rows = np.concatenate([np.full(len(b), k, np.int64) for k, b in enumerate(blocks)])
    cols = np.concatenate(blocks)
    Mem = sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(nb, n))
    G = A.tocsr().copy()
    G.data = np.ones_like(G.data)
    G = (G + sp.identity(n, format='csr')).tocsr()
    G.data[:] = 1.0
    C = (Mem @ (Mem @ G).T).tocsr()
    colour = np.full(nb, -1, np.int64)
    for k in range(nb):
        nb_k = C.indices[C.indptr[k]:C.indptr[k + 1]]
        used = set(colour[nb_k[nb_k < k]].tolist())
        c = 0
        while c in used:
            c += 1
        colour[k] = c
    return colour.astype(np.int32)


class Rings:
    """Level-0 seed-ring blocks (Schwarz_type RINGS): members sorted per block
    (seed_ring_blocks), Gauss-Jordan inverses, greedy conflict colouring."""

    def __init__(self, A: sp.csr_matrix, seeds, maxlvl: int, mmsize: int):
        A = A.tocsr()
        n = A.shape[0]
        seeds = np.asarray(seeds, np.int64)
        if seeds.size == 0:
            raise ValueError('seed-ring Schwarz needs seeds')
        if float(seeds.size) * mmsize * mmsize > 4e9:
            raise ValueError('seed-ring Schwarz (dense overlapping blocks) is for sparse seed sets')
        self.blocks = seed_ring_blocks(A, seeds, maxlvl, mmsize)
        self.Minv = [batched_inverse(A[b][:, b].toarray()[None, :, :])[0] for b in self.blocks]
        self.colour = ring_colouring(A, self.blocks)
        self.ncolours = int(self.colour.max()) + 1
        self.cblocks = [np.flatnonzero(self.colour == c) for c in range(self.ncolours)]
        self.cov = np.zeros(n, dtype=bool)
        for b in self.blocks:
            self.cov[b] = True
        self.seed_order = False      # True: sweep_seed_order (HAZmath's order) in the cycle

    def sweep_seed_order(self, A: sp.csr_matrix, x: np.ndarray, b: np.ndarray, forward=True):
        """HAZmath's order (SCHWARZ_SYMMETRIC, recalled): the blocks one at a
        time in seed order (forward) or reverse seed order (backward), each
        block's residual taken after every earlier block's update.  The GPU
        runs the colour order of ``sweep`` instead (a substitution: the same
        blocks and local solves, another multiplicative order); this one is
        the oracle's reference for that difference (tests/test_rings_oracle.py)."""
        ks = range(len(self.blocks)) if forward else range(len(self.blocks) - 1, -1, -1)
        A = A.tocsr()
        for k in ks:
            blk = self.blocks[k]
            x[blk] += self.Minv[k] @ (b[blk] - A[blk] @ x)
        return x

    def sweep(self, A: sp.csr_matrix, x: np.ndarray, b: np.ndarray, forward=True):
        """x <- x + Minv_k (b - A x)|_k for the blocks of each colour in turn
        (ascending if forward, else descending); blocks of one colour are
        independent, so their residuals are taken before any of them updates."""
        order = range(self.ncolours) if forward else range(self.ncolours - 1, -1, -1)
        for c in order:
            ks = self.cblocks[c]
            rows = np.concatenate([self.blocks[k] for k in ks])
            res = b[rows] - A[rows] @ x
            off = 0
            for k in ks:
                m = len(self.blocks[k])
                x[self.blocks[k]] += self.Minv[k] @ res[off:off + m]
                off += m
        return x


def rest_gs_inverse(A: sp.csr_matrix, cov: np.ndarray) -> np.ndarray:
    """(nv, 2, 2) node-block inverses of the rest Gauss-Seidel: both dofs of
    node I uncovered -> the 2x2 Gauss-Jordan inverse of A's diagonal block
    (node_block_inverse); one uncovered dof f -> 1 / a_ff at (f, f); covered
    dofs -> 0 (no update)."""
    n = A.shape[0]
    nv = n // 2
    Dn = node_block_inverse(A, np.arange(n) % nv, nv)
    d = A.diagonal()
    c0, c1 = cov[:nv], cov[nv:]
    half0 = ~c0 & c1                      # only field 0 uncovered
    half1 = c0 & ~c1
    Dn[c0 | c1] = 0.0
    Dn[half0, 0, 0] = 1.0 / d[:nv][half0]
    Dn[half1, 1, 1] = 1.0 / d[nv:][half1]
    return Dn


@dataclasses.dataclass
class Level:
    A: sp.csr_matrix
    winv: np.ndarray = None          # point smoother weights (vector)
    WB: sp.csr_matrix = None         # block smoother (level 0 with seeds)
    P: sp.csr_matrix = None
    R: sp.csr_matrix = None
    agg: np.ndarray = None
    nagg: int = 0
    w_sa: float = 0.0
    Ainv: np.ndarray = None
    bid: np.ndarray = None
    colour: np.ndarray = None        # multicolour GS: colour per node
    ncolours: int = 0
    Dn: np.ndarray = None            # multicolour GS: (nv, 2, 2) block inverses
    crows: list = None               # node ids of each colour (ascending)
    polyW: list = None               # POLY: w_k W per Chebyshev step (poly_weights)
    patches: 'Patches' = None        # level 0, Schwarz_type PATCHES
    rings: 'Rings' = None            # level 0, Schwarz_type RINGS (Dn / colour: the rest GS)

    def step_smoother(self, k):
        return None if self.polyW is None else self.polyW[k]

    def smooth_apply(self, r, S=None):
        if S is None:
            return self.WB @ r if self.WB is not None else self.winv * r
        return S @ r if sp.issparse(S) else S * r

    def gs_sweep(self, x, b, forward=True):
        """x <- x + D_I^-1 (b - A x)_I for the nodes I of each colour in turn
        (colours ascending if forward, else descending); nodes of one colour
        are never adjacent, so each colour step is one parallel update."""
        nv = self.A.shape[0] // 2
        order = range(self.ncolours) if forward else range(self.ncolours - 1, -1, -1)
        for c in order:
            I = self.crows[c]
            rows = np.concatenate([I, nv + I])
            res = b[rows] - self.A[rows] @ x
            r0, r1 = res[:len(I)], res[len(I):]
            D = self.Dn[I]
            x[I] = x[I] + (D[:, 0, 0] * r0 + D[:, 0, 1] * r1)
            x[nv + I] = x[nv + I] + (D[:, 1, 0] * r0 + D[:, 1, 1] * r1)
        return x


class Hierarchy:
    def __init__(self, levels, params):
        self.levels = levels
        self.params = params

    # ---------------------------------------------------------------- apply
    def cycle(self, l: int, b: np.ndarray) -> np.ndarray:
        """Multigrid cycle from a zero initial guess (V, or W: the coarse
        problem is visited twice, 2nd visit on the updated residual)."""
        p = self.params
        lev = self.levels[l]
        if lev.Ainv is not None:
            return lev.Ainv @ b
        A = lev.A
        gs = lev.colour is not None
        if lev.rings is not None:                    # seed-ring Schwarz + the rest's GS (symmetric step)
            x = np.zeros_like(b)
            for _ in range(p.presmooth_iter):
                x = self.rings_step(lev, x, b)
        elif lev.patches is not None:                # symmetric multiplicative patch Schwarz
            x = np.zeros_like(b)
            for _ in range(p.presmooth_iter):
                x = lev.patches.sweep(A, x, b, True)
                x = lev.patches.sweep(A, x, b, False)
        elif gs:                                     # SGS: forward + backward; GS: forward
            x = np.zeros_like(b)
            for _ in range(p.presmooth_iter):
                x = lev.gs_sweep(x, b, True)
                if p.smoother == 'SGS':
                    x = lev.gs_sweep(x, b, False)
        else:
            # step smoothers: [W] * nu1 (Jacobi), [w_1 W .. w_m W] * nu1 (POLY)
            pre = [None] * p.presmooth_iter
            if lev.polyW is not None:
                pre = lev.polyW * p.presmooth_iter
            x = lev.smooth_apply(b, pre[0])          # first sweep from x = 0
            for S in pre[1:]:
                x = x + lev.smooth_apply(b - A @ x, S)
        r = b - A @ x
        bc = lev.R @ r
        C = self.levels[l + 1]
        e = self.cycle(l + 1, bc)
        if p.cycle_type == 'W' and C.Ainv is None:
            e = e + self.cycle(l + 1, bc - C.A @ e)
        if p.coarse_scaling:                         # src/amg_parameters.py:78
            e = coarse_scale(C.A, bc, e)
        x = x + lev.P @ e
        post = [None]
        if lev.polyW is not None:
            post = lev.polyW[::-1]                   # POLY: steps m..1
        for _ in range(p.postsmooth_iter):
            if lev.rings is not None:
                x = self.rings_step(lev, x, b)
            elif lev.patches is not None:
                x = lev.patches.sweep(A, x, b, True)
                x = lev.patches.sweep(A, x, b, False)
            elif gs:                                 # SGS: forward + backward; GS: backward
                if p.smoother == 'SGS':
                    x = lev.gs_sweep(x, b, True)
                x = lev.gs_sweep(x, b, False)
            else:
                for S in post:
                    x = x + lev.smooth_apply(b - A @ x, S)
        return x

    @staticmethod
    def rings_step(lev, x, b):
        """One symmetric level-0 step of Schwarz_type RINGS: ring sweep
        forward, rest GS forward and backward, ring sweep backward."""
        sw = lev.rings.sweep_seed_order if lev.rings.seed_order else lev.rings.sweep
        x = sw(lev.A, x, b, True)
        x = lev.gs_sweep(x, b, True)
        x = lev.gs_sweep(x, b, False)
        return sw(lev.A, x, b, False)

    def apply(self, r: np.ndarray) -> np.ndarray:
        """z = B r: ``maxit`` cycles (src/amg_parameters.py:71), x0 = 0."""
        z = self.cycle(0, r)
        A0 = self.levels[0].A
        for _ in range(self.params.maxit - 1):
            z = z + self.cycle(0, r - A0 @ z)
        return z

    def __call__(self, r):
        return self.apply(r)

    def info(self):
        return [(lv.A.shape[0], lv.A.nnz, 0 if lv.P is None else lv.P.nnz)
                for lv in self.levels]


def coarse_scale(Ac, bc, e):
    """Coarse-grid correction scaling (HAZmath `coarse_scaling: ON`,
    src/amg_parameters.py:78): the fine correction P e is scaled by
    alpha = <r, P e> / <A P e, P e>.  With R = P^T and A_c = R A P (Galerkin)
    this is <b_c, e> / <A_c e, e>, computed on the coarse level; alpha = 1 if
    the denominator is not positive."""
    q = Ac @ e
    den = float(np.dot(e, q))
    alpha = float(np.dot(bc, e)) / den if den > 0 else 1.0
    return alpha * e


SCHWARZ_SYMMETRIC = 3
SCHWARZ_SEED_BLOCKS = 7        # the level smoother on non-overlapping seed blocks


def resolve_params(p: Params, idofs=None, n: int = 0) -> Params:
    """The reference's SCHWARZ_SYMMETRIC on the seeds' overlapping
    seed + Schwarz_maxlvl ring blocks (src/amg_parameters.py:83-87,
    src/utils.py:60-86) of a nodal system; mirrors setup.cpp resolve_params:
    * no seeds: no Schwarz level (the level smoother everywhere);
    * 1-rings with a seed on every node: the node patches (SCHWARZ_PATCHES,
      the same blocks, a dedicated kernel);
    * otherwise: the seed rings (SCHWARZ_RINGS)."""
    if p.Schwarz_levels >= 1 and p.Schwarz_type == SCHWARZ_SYMMETRIC and p.Schwarz_maxlvl >= 1 \
            and p.num_functions == 2 and p.node_block_smoother:
        if idofs is None or len(idofs) == 0:
            return dataclasses.replace(p, Schwarz_levels=0)
        nv = n // 2
        every = p.Schwarz_maxlvl == 1 and n > 0 and \
            np.unique(np.asarray(idofs, np.int64) % nv).size == nv
        return dataclasses.replace(p, Schwarz_type=SCHWARZ_PATCHES if every else SCHWARZ_RINGS)
    return p



AGGREGATORS = {'MIS': aggregate_mis2, 'HEM': aggregate_hem, 'VMB': aggregate_vmb}


def setup(A: sp.csr_matrix, params: Params | None = None, idofs=None) -> Hierarchy:
    p = resolve_params(params or Params(), idofs, A.shape[0])
    A = A.tocsr()
    A.sort_indices()
    levels = []
    cur = A
    for l in range(p.max_levels):
        lev = Level(A=cur)
        levels.append(lev)
        n = cur.shape[0]
        last = (n <= p.coarse_dof) or (l == p.max_levels - 1)
        nf = p.num_functions
        if not last:
            if nf > 1:
                S, Wn = node_strength(cur, nf, p.strong_coupled, p.strength_measure)
                agg, nagg = AGGREGATORS[p.aggregation_type](Wn, S, l)
                last = nagg == 0 or nf * nagg >= n
            else:
                S = strength(cur, p.strong_coupled, p.strength_measure)
                agg, nagg = AGGREGATORS[p.aggregation_type](abs(cur), S, l)
                last = nagg == 0 or nagg >= n
        if last:
            if n > p.max_coarse_dense:
                raise RuntimeError('coarsest level %d too large for dense solve' % n)
            lev.Ainv = dense_inverse(cur.toarray())
            break
        gs = p.smoother in ('SGS', 'GS')
        if gs and (nf != 2 or not p.node_block_smoother):
            raise ValueError('multicolour GS needs num_functions = 2 and node-block smoothers')
        pj = dataclasses.replace(p, smoother='JACOBI_RHO') if gs else p
        rings = l == 0 and p.Schwarz_levels >= 1 and p.Schwarz_type == SCHWARZ_RINGS and idofs is not None
        if rings and (nf != 2 or not p.node_block_smoother):
            raise ValueError('seed-ring Schwarz needs num_functions = 2 and node-block smoothers')
        if rings:                                    # node blocks (the level-0 W is not applied)
            lev.WB, lev.bid, nbk = block_smoother(cur, None, pj, node_blocks(n, nf))
        elif l < p.Schwarz_levels and idofs is not None and l == 0 and p.Schwarz_maxlvl >= 1 \
                and p.Schwarz_type == SCHWARZ_ADDITIVE:
            lev.WB, _ = overlap_smoother(cur, idofs, pj)
            nbk = 0
        elif l < p.Schwarz_levels and idofs is not None and l == 0 and p.Schwarz_maxlvl >= 1:
            lev.WB, lev.bid, nbk = block_smoother(cur, idofs, pj)
        elif nf > 1 and p.node_block_smoother:
            lev.WB, lev.bid, nbk = block_smoother(cur, None, pj, node_blocks(n, nf))
        else:
            lev.winv = smoother_weights(cur, p)
        if p.smoother == 'POLY':
            lev.polyW = [scaled_smoother(lev, w) for w in poly_weights(p)]
        if gs:
            lev.Dn = node_block_inverse(cur, lev.bid, nbk)
            lev.colour = jp_colouring(node_pattern(cur, 2), l)
            lev.ncolours = int(lev.colour.max()) + 1 if len(lev.colour) else 0
            lev.crows = [np.flatnonzero(lev.colour == c) for c in range(lev.ncolours)]
        if rings:
            lev.rings = Rings(cur, idofs, p.Schwarz_maxlvl, p.Schwarz_mmsize)
            lev.Dn = rest_gs_inverse(cur, lev.rings.cov)
            lev.colour = jp_colouring(node_pattern(cur, 2), l)
            lev.ncolours = int(lev.colour.max()) + 1 if len(lev.colour) else 0
            lev.crows = [np.flatnonzero(lev.colour == c) for c in range(lev.ncolours)]
        if l == 0 and p.Schwarz_levels >= 1 and p.Schwarz_type == SCHWARZ_PATCHES:
            if nf != 2 or p.Schwarz_maxlvl != 1:
                raise ValueError('node patches need num_functions = 2 and Schwarz_maxlvl = 1')
            lev.patches = Patches(cur, idofs)
        lev.agg, lev.nagg = agg, nagg
        T = tentative_nodal(agg, nagg, nf) if nf > 1 else tentative(agg, nagg)
        if p.AMG_type == 'SA':
            if nf > 1 and p.sa_block_diag:
                P, lev.w_sa = smooth_prolongator_block(cur, T, p.sa_omega, node_blocks(n, nf))
            else:
                P, lev.w_sa = smooth_prolongator(cur, T, p.sa_omega, p.rho_iters)
        elif p.AMG_type == 'UA':
            P = T
        else:
            raise ValueError(p.AMG_type)
        lev.P = P
        lev.R, cur = galerkin(cur, P)
    return Hierarchy(levels, p)


# --------------------------------------------------------------------------
# PCG, cbc.block ``cgN`` semantics [ext, recalled]
# --------------------------------------------------------------------------
class CGResult:
    def __init__(self, x, residuals, alphas, betas):
        self.x, self.residuals, self.alphas, self.betas = x, residuals, alphas, betas

    @property
    def niters(self):
        return len(self.residuals) - 1

    def eigenvalue_estimates(self):
        return lanczos_eigs(self.alphas, self.betas)


def pcg(A, B, b, tolerance=1e-8, maxiter=500, x0=None, relativeconv=False):
    """r = b - A x; z = B r; d = z; rz = <r,z>; residuals = [sqrt(rz)];
    while residuals[-1] > tol and iter < maxiter: ... (cbc.block cgN)."""
    x = np.zeros_like(b) if x0 is None else x0.copy()
    r = b - A @ x
    z = B(r)
    d = z.copy()
    rz = float(np.dot(r, z))
    if rz < 0:
        raise ValueError('Matrix is not positive')
    residuals = [np.sqrt(rz)]
    alphas, betas = [], []
    tol = tolerance * residuals[0] if relativeconv else tolerance
    it = 0
    while residuals[-1] > tol and it < maxiter:
        z = A @ d
        dz = float(np.dot(d, z))
        if dz == 0:
            break
        alpha = rz / dz
        x = x + alpha * d
        r = r - alpha * z
        z = B(r)
        rz_prev = rz
        rz = float(np.dot(r, z))
        if rz < 0:
            x = x - alpha * d
            break
        beta = rz / rz_prev
        d = z + beta * d
        residuals.append(np.sqrt(rz))
        alphas.append(alpha)
        betas.append(beta)
        it += 1
    return CGResult(x, residuals, alphas, betas)


def lanczos_eigs(alphas, betas):
    """Eigenvalues of the CG Lanczos tridiagonal: T00 = 1/a0,
    Tkk = 1/ak + b(k-1)/a(k-1), T(k,k-1) = sqrt(b(k-1))/a(k-1)."""
    n = len(alphas)
    if n == 0:
        return np.array([1.0])
    T = np.zeros((n, n))
    T[0, 0] = 1.0 / alphas[0]
    for k in range(1, n):
        T[k, k] = 1.0 / alphas[k] + betas[k - 1] / alphas[k - 1]
        T[k, k - 1] = np.sqrt(betas[k - 1]) / alphas[k - 1]
        T[k - 1, k] = T[k, k - 1]
    e = np.linalg.eigvalsh(T)
    return np.sort(e)


def seeded_rhs(N: int, seed: int = 1234) -> np.ndarray:
    """uniform(-1,1) fp64 from numpy's default_rng(seed)."""
    return np.random.default_rng(seed).uniform(-1.0, 1.0, N)
