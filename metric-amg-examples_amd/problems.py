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


def finest_n(dim: int, nrefs: int, problem: str = 'bidomain') -> int:
    """Finest mesh of the drivers' refinement loops: bidomain_2d/3d
    2**(5|3 + nrefs - 1) (src/bidomain_2d.py:168, src/bidomain_3d.py:113),
    emi_2d/3d 2**(6|2 + nrefs - 1) (src/emi_2d.py:190, src/emi_3d.py:119)."""
    first = {('bidomain', 2): 5, ('bidomain', 3): 3, ('emi', 2): 6, ('emi', 3): 2}[(problem, dim)]
    return 2 ** (first + nrefs - 1)


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


@dataclasses.dataclass
class SystemMeta:
    """Sizes and seeds of a bidomain system whose matrix lives elsewhere (in
    HBM, bidomain_device): what a multi-GPU rank needs on the host."""
    N: int
    nv: int
    dim: int
    n: int
    nnz: int

    @property
    def idofs(self) -> np.ndarray:
        return np.arange(self.nv, 2 * self.nv, dtype=np.int32)

    @property
    def W(self):
        return [self.nv, self.nv]


def bidomain_meta(dim: int, n: int, nnz: int) -> SystemMeta:
    nv = (n + 1) ** dim
    return SystemMeta(2 * nv, nv, dim, n, int(nnz))


def bidomain_device(dim: int, n: int, gamma: float, kappa1: float = 2.0, kappa2: float = 3.0, device=None):
    """The same matrix as ``bidomain`` built in HBM by the gfx950 generator
    (mamg_gen_bidomain_device, bitwise the host generator's): a tuple of CUDA
    tensors (indptr int64, indices int32, data float64) for MetricAMG /
    DistMetricAMG, so a rank of a multi-GPU job never holds the global matrix
    on the host."""
    import ctypes as C
    import torch
    L = _lib.lib()
    N, nnz = C.c_int64(), C.c_int64()
    _lib.check(L.mamg_gen_bidomain_size(dim, n, C.byref(N), C.byref(nnz)))
    dev = torch.device('cuda', torch.cuda.current_device()) if device is None else torch.device(device)
    ip = torch.empty(N.value + 1, dtype=torch.int64, device=dev)
    ix = torch.empty(nnz.value, dtype=torch.int32, device=dev)
    dv = torch.empty(nnz.value, dtype=torch.float64, device=dev)
    torch.cuda.synchronize(dev)
    with torch.cuda.device(dev):
        _lib.check(L.mamg_gen_bidomain_device(dim, n, gamma, kappa1, kappa2, nnz.value, C.c_void_p(ip.data_ptr()),
                                              C.c_void_p(ix.data_ptr()), C.c_void_p(dv.data_ptr())))
    return ip, ix, dv


def bidomain_mms_rhs(dim: int, n: int, gamma: float, kappa1: float = 2.0, kappa2: float = 3.0) -> np.ndarray:
    """Right-hand side of bidomain(dim, n, ...) for the reference's manufactured
    solution (src/bidomain_2d.py:7-99, src/bidomain_3d.py:7-49; csrc/mms.cpp)."""
    L = _lib.lib()
    N, nnz = C.c_int64(), C.c_int64()
    _lib.check(L.mamg_gen_bidomain_size(dim, n, C.byref(N), C.byref(nnz)))
    b = np.empty(N.value, dtype=np.float64)
    _lib.check(L.mamg_gen_bidomain_mms(dim, n, float(gamma), float(kappa1), float(kappa2),
                                       _lib.ptr(b, C.c_double)))
    return b


def bidomain_mms_errors(dim: int, n: int, x, gamma: float, kappa1: float = 2.0, kappa2: float = 3.0):
    """(|u1 - u1h|_H1, |u2 - u2h|_H1) of a solution x of the manufactured problem
    (errornorm(u, uh, 'H1'), src/bidomain_2d.py:239-240)."""
    L = _lib.lib()
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    nv = (n + 1) ** dim
    if x.shape != (2 * nv,):
        raise ValueError('x must have 2 (n+1)^dim entries')
    err = np.zeros(2)
    _lib.check(L.mamg_bidomain_mms_error(dim, n, float(gamma), float(kappa1), float(kappa2),
                                         _lib.ptr(x, C.c_double), _lib.ptr(err, C.c_double)))
    return float(err[0]), float(err[1])


def seeded_rhs(N: int, seed: int = 1234) -> np.ndarray:
    """uniform(-1, 1) fp64, numpy default_rng(seed)."""
    return np.random.default_rng(seed).uniform(-1.0, 1.0, N)


# ---------------------------------------------------------------------------
# P1 on boxes of dolfin's structured simplices (EMI halves, the 3D-1D tissue).
# dolfin's UnitSquareMesh 'right' / UnitCubeMesh split every cell into the
# monotone lattice paths from its lower to its upper corner, so the element
# matrices of one simplex are the path matrices below (K: stiffness, M: mass).
# ---------------------------------------------------------------------------
_PATH_K = {2: np.array([[1, -1, 0], [-1, 2, -1], [0, -1, 1]], np.float64) / 2.0,
           3: np.array([[1, -1, 0, 0], [-1, 2, -1, 0], [0, -1, 2, -1], [0, 0, -1, 1]], np.float64) / 6.0}


def _simplices(cells: np.ndarray, dim: int) -> list:
    """Vertex lattice coordinates (list over simplex vertices of [ncell, dim]
    int arrays) of every path simplex of the given lower-corner cells."""
    import itertools
    out = []
    for path in itertools.permutations(range(dim)):
        verts = [cells.copy()]
        cur = cells.copy()
        for ax in path:
            cur = cur.copy()
            cur[:, ax] += 1
            verts.append(cur)
        out.append(verts)
    return out


def _assemble(simplices, index, nv, Kloc, Mloc):
    """Sum element matrices into CSR (K, M) over vertex numbering `index`."""
    import scipy.sparse as sp
    rows, cols, kv, mv = [], [], [], []
    for verts in simplices:
        ids = [index(v) for v in verts]
        for a in range(len(ids)):
            for b in range(len(ids)):
                rows.append(ids[a]); cols.append(ids[b])
                kv.append(np.full(len(ids[a]), Kloc[a, b]))
                mv.append(np.full(len(ids[a]), Mloc[a, b]))
    r, c = np.concatenate(rows), np.concatenate(cols)
    K = sp.coo_matrix((np.concatenate(kv), (r, c)), shape=(nv, nv)).tocsr()
    M = sp.coo_matrix((np.concatenate(mv), (r, c)), shape=(nv, nv)).tocsr()
    K.sort_indices(); M.sort_indices()
    return K, M


def _mass_loc(d: int, meas: float) -> np.ndarray:
    """P1 mass matrix of a d-simplex of measure meas: meas/((d+1)(d+2)) (1 + I)."""
    return meas / ((d + 1) * (d + 2)) * (np.ones((d + 1, d + 1)) + np.eye(d + 1))


@dataclasses.dataclass
class BlockSystem:
    """2x2 block system [[A00, A01], [A10, A11]] with its monolithic CSR
    (ii_convert order [u0; u1]) and the reference driver's interface dofs."""
    blocks: list              # [[A00, A01], [A10, A11]] scipy CSR
    W: list                   # [dim V0, dim V1]
    idofs: np.ndarray         # interface / seed dofs (monolithic numbering)
    name: str = ''
    info: dict = dataclasses.field(default_factory=dict)

    def scipy(self):
        import scipy.sparse as sp
        A = sp.bmat(self.blocks, format='csr')
        A.sort_indices()
        return A

    @property
    def N(self):
        return int(sum(self.W))

    @property
    def nv(self):
        """dofs per field when both blocks have the same size (EMI: mirror-image
        numbering, so dof I of each side forms node I of a 2-field system)."""
        if self.W[0] != self.W[1]:
            raise ValueError('blocks of different sizes: no node pairing')
        return int(self.W[0])

    def tocsr(self):
        if self.info.get('_csr') is None:
            self.info['_csr'] = self.scipy()
        return self.info['_csr']

    @property
    def nnz(self):
        return int(self.tocsr().nnz)


def _eliminate(A, dofs):
    """Symmetric Dirichlet elimination (rows and columns of `dofs` -> unit diagonal)."""
    import scipy.sparse as sp
    keep = np.ones(A.shape[0])
    keep[dofs] = 0.0
    D = sp.diags(keep)
    A = (D @ A @ D + sp.diags(1.0 - keep)).tocsr()
    A.eliminate_zeros()
    A.sort_indices()
    return A


def emi(dim: int, n: int, gamma: float, kappa1: float = 2.0, kappa2: float = 3.0,
        both_sides: bool | None = None) -> BlockSystem:
    """EMI primal system on the split unit square / cube (src/emi_2d.py:58-128,
    meshes src/utils.py:187-260): Omega_1 = {x_d > 1/2} (tag-1 cells),
    Omega_2 = {x_d < 1/2}, each with its own P1 space; coupled on the interface
    Gamma = {x_d = 1/2} by the trace terms

        a00 = k1 K_1 + g T1' M_G T1      a01 = -g T1' M_G T2
        a10 = -g T2' M_G T1              a11 = k2 K_2 + g T2' M_G T2

    (src/emi_2d.py:86-89).  Dirichlet: u1 on x_d = 1 (tag 3), u2 on x_d = 0
    (tag 6) (:108-111), eliminated symmetrically.  Vertex numbering of each
    half is (layer distance from Gamma, then lattice order), so dof I of u1 and
    dof I of u2 are mirror images; interface dofs: the u1 side in 2-D
    (src/emi_2d.py:205-206), both sides in 3-D (src/emi_3d.py:134-138) unless
    both_sides says otherwise."""
    import scipy.sparse as sp
    if n < 4 or n % 2:
        raise ValueError('n must be even and >= 4')
    h = 1.0 / n
    m = n // 2
    vert_shape = [n + 1] * (dim - 1) + [m + 1]
    nv = int(np.prod(vert_shape))

    def half(top: bool):
        cells, index = emi_half(dim, n, top)
        Kloc = _PATH_K[dim] * (h if dim == 3 else 1.0)
        Mloc = _mass_loc(dim, h ** dim / (2 if dim == 2 else 6))
        return _assemble(_simplices(cells, dim), index, nv, Kloc, Mloc)[0]

    K1, K2 = half(True), half(False)
    # interface mass: (dim-1)-simplices of the plane x_d = 1/2 (layer 0 of both halves)
    ng = (n + 1) ** (dim - 1)
    if dim == 2:
        s = np.arange(n)
        segs = [s, s + 1]
        MG = _assemble_simplices_flat(segs, ng, _mass_loc(1, h))
    else:
        i, j = np.meshgrid(np.arange(n), np.arange(n), indexing='ij')
        i, j = i.ravel(), j.ravel()
        v = lambda a, b: (j + b) * (n + 1) + (i + a)
        tris = [[v(0, 0), v(1, 0), v(1, 1)], [v(0, 0), v(0, 1), v(1, 1)]]
        MG = sum(_assemble_simplices_flat(t, ng, _mass_loc(2, h * h / 2)) for t in tris)
    T = sp.csr_matrix((np.ones(ng), (np.arange(ng), np.arange(ng))), shape=(ng, nv))
    C = (T.T @ MG @ T).tocsr()
    A00 = (kappa1 * K1 + gamma * C).tocsr()
    A11 = (kappa2 * K2 + gamma * C).tocsr()
    A01 = (-gamma * C).tocsr()
    outer = np.arange(nv - ng, nv)             # last layer: x_d = 1 (u1) / x_d = 0 (u2)
    A = sp.bmat([[A00, A01], [A01.T, A11]], format='csr')
    A = _eliminate(A, np.concatenate([outer, nv + outer]))
    blocks = [[A[:nv, :nv].tocsr(), A[:nv, nv:].tocsr()], [A[nv:, :nv].tocsr(), A[nv:, nv:].tocsr()]]
    if both_sides is None:
        both_sides = dim == 3
    gam = np.arange(ng, dtype=np.int32)
    idofs = np.concatenate([gam, nv + gam]) if both_sides else gam
    return BlockSystem(blocks, [nv, nv], idofs.astype(np.int32), 'emi_%dd' % dim,
                       dict(dim=dim, n=n, gamma=gamma, kappa1=kappa1, kappa2=kappa2, n_interface=ng))


def emi_half(dim: int, n: int, top: bool):
    """(lower-corner lattice coordinates of the half's cells, vertex -> dof
    index) of Omega_1 (top, x_d > 1/2) or Omega_2: dofs numbered by layer
    distance from Gamma, then lattice order (problems.emi)."""
    m = n // 2
    grids = np.meshgrid(*[np.arange(s) for s in [n] * (dim - 1) + [m]], indexing='ij')
    cells = np.stack([g.ravel() for g in grids], axis=1).astype(np.int64)
    cells[:, dim - 1] += m if top else 0         # global lattice layer of the cell's lower corner

    def index(v):
        layer = v[:, dim - 1] - m if top else m - v[:, dim - 1]
        idx = layer
        for d in range(dim - 2, -1, -1):
            idx = idx * (n + 1) + v[:, d]
        return idx
    return cells, index


def _assemble_simplices_flat(ids, nv, Mloc):
    import scipy.sparse as sp
    rows, cols, vals = [], [], []
    for a in range(len(ids)):
        for b in range(len(ids)):
            rows.append(ids[a]); cols.append(ids[b]); vals.append(np.full(len(ids[a]), Mloc[a, b]))
    M = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(nv, nv)).tocsr()
    M.sort_indices()
    return M


def neuron_curve(n: int):
    """Synthetic stand-in for the neuron centreline mesh of src/emi_3d1d.py:28-43
    (PolyIC_3AS2_1.CNG.c1.h5, downloaded from Google Drive: unavailable
    offline).  A branched polyline made of edges of the 3-D mesh (as
    EmbeddedMesh(edge_f, 1) is): a soma-to-axon trunk along x through the
    cube centre, one dendrite along the cells' body diagonal (1,1,1) and one
    along +y from the branch point.  Returns (lattice points [m,3], edges [e,2])."""
    c = n // 2
    q = max(2, n // 8)
    pts, edges = [], []
    index = {}

    def add(p):
        p = tuple(int(t) for t in p)
        if p not in index:
            index[p] = len(pts)
            pts.append(p)
        return index[p]

    def walk(start, step, count):
        a = add(start)
        p = np.array(start)
        for _ in range(count):
            p = p + np.array(step)
            b = add(p)
            edges.append((a, b))
            a = b

    walk((q, c, c), (1, 0, 0), n - 2 * q)                 # trunk
    walk((c, c, c), (1, 1, 1), (n - 2 * q) // 3)          # dendrite 1
    walk((c, c, c), (0, 1, 0), (n - 2 * q) // 2)          # dendrite 2
    return np.array(pts, np.int64), np.array(edges, np.int64)


def _p1_eval_weights(x: np.ndarray, n: int):
    """P1 basis weights of the structured cube mesh (h = 1 lattice units) at
    points x [k,3]: returns (vertex ids [k,4], weights [k,4]).  The simplex
    containing a point of cell c with local coordinates a is the path through
    the axes sorted by decreasing a."""
    x = np.clip(x, 0.0, n - 1e-12)
    cell = np.floor(x).astype(np.int64)
    a = x - cell
    order = np.argsort(-a, axis=1, kind='stable')
    asrt = np.take_along_axis(a, order, axis=1)
    w = np.stack([1.0 - asrt[:, 0], asrt[:, 0] - asrt[:, 1], asrt[:, 1] - asrt[:, 2], asrt[:, 2]], axis=1)
    verts = [cell.copy()]
    cur = cell.copy()
    for k in range(3):
        cur = cur.copy()
        np.add.at(cur, (np.arange(len(cur)), order[:, k]), 1)
        verts.append(cur)
    nn = n + 1
    ids = np.stack([(v[:, 2] * nn + v[:, 1]) * nn + v[:, 0] for v in verts], axis=1)
    return ids, w


def emi_3d1d(n: int, gamma: float, radius: float = 1.0, quad: int = 16) -> BlockSystem:
    """Reduced 3D-1D EMI system of src/emi_3d1d.py:46-94 on a synthetic
    neuron (``neuron_curve``) in the cube [0, n]^3 micrometres (h = 1 um,
    the scale of the reference's neuron mesh).  Parameters as the driver sets
    them (:125-134): sigma3 = 3, sigma1 = 7 pi rho^2 (7 pi if rho = 0),
    gamma_c = dt^-1 * 2 pi rho C_m (2 pi if rho = 0), C_m = 1, dt^-1 = gamma.

        a00 = k3 (K3 + M3) + g Avg' M1 Avg      a01 = -g Avg' M1
        a10 = -g M1 Avg                         a11 = k1 (K1 + M1) + g M1

    Avg = trace on the curve (rho = 0) or the mean over the circle of radius
    rho normal to the curve (``quad`` points; xii's Average with
    Circle(radius)), P1-interpolated.  Homogeneous Neumann everywhere.  Seeds:
    the 1D dofs, as utils.dump_system writes them (src/utils.py:321)."""
    import scipy.sparse as sp
    mc = 1.0
    sigma3 = 3.0
    if radius > 0:
        gc = gamma * 2 * np.pi * radius * mc
        sigma1 = 7.0 * np.pi * radius ** 2
    else:
        gc = gamma * 2 * np.pi * mc
        sigma1 = 7.0 * np.pi
    nn = n + 1
    nv3 = nn ** 3
    grids = np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing='ij')
    cells = np.stack([g.ravel() for g in grids], axis=1).astype(np.int64)
    idx3 = lambda v: (v[:, 2] * nn + v[:, 1]) * nn + v[:, 0]
    K3, M3 = _assemble(_simplices(cells, 3), idx3, nv3, _PATH_K[3], _mass_loc(3, 1.0 / 6))
    pts, edges = neuron_curve(n)
    nq = len(pts)
    L = np.linalg.norm(pts[edges[:, 1]] - pts[edges[:, 0]], axis=1).astype(np.float64)
    ids = [edges[:, 0], edges[:, 1]]
    rows, cols, kv, mv = [], [], [], []
    for a in range(2):
        for b in range(2):
            rows.append(ids[a]); cols.append(ids[b])
            kv.append((1.0 if a == b else -1.0) / L)
            mv.append(L / 6.0 * (2.0 if a == b else 1.0))
    r, c = np.concatenate(rows), np.concatenate(cols)
    K1 = sp.coo_matrix((np.concatenate(kv), (r, c)), shape=(nq, nq)).tocsr()
    M1 = sp.coo_matrix((np.concatenate(mv), (r, c)), shape=(nq, nq)).tocsr()
    # averaging operator Avg [nq, nv3]
    tang = np.zeros((nq, 3))
    for e in edges:
        d = pts[e[1]] - pts[e[0]]
        d = d / np.linalg.norm(d)
        for v in e:
            if not tang[v].any():
                tang[v] = d
    if radius > 0:
        helper = np.where(np.abs(tang[:, :1]) < 0.9, np.array([[1.0, 0, 0]]), np.array([[0, 1.0, 0]]))
        n1 = np.cross(tang, helper)
        n1 /= np.linalg.norm(n1, axis=1, keepdims=True)
        n2 = np.cross(tang, n1)
        th = 2 * np.pi * np.arange(quad) / quad
        X = (pts[:, None, :] + radius * (np.cos(th)[None, :, None] * n1[:, None, :]
                                         + np.sin(th)[None, :, None] * n2[:, None, :])).reshape(-1, 3)
        vid, w = _p1_eval_weights(X, n)
        qrow = np.repeat(np.arange(nq), quad * 4)
        Avg = sp.coo_matrix((w.ravel() / quad, (qrow, vid.ravel())), shape=(nq, nv3)).tocsr()
    else:
        Avg = sp.csr_matrix((np.ones(nq), (np.arange(nq), idx3(pts))), shape=(nq, nv3))
    Avg.sum_duplicates()
    A00 = (sigma3 * (K3 + M3) + gc * (Avg.T @ M1 @ Avg)).tocsr()
    A01 = (-gc * (Avg.T @ M1)).tocsr()
    A10 = (-gc * (M1 @ Avg)).tocsr()
    A11 = (sigma1 * (K1 + M1) + gc * M1).tocsr()
    blocks = [[A00, A01], [A10, A11]]
    for row in blocks:
        for B in row:
            B.sort_indices()
    idofs = np.arange(nv3, nv3 + nq, dtype=np.int32)
    return BlockSystem(blocks, [nv3, nq], idofs, 'emi_3d1d',
                       dict(n=n, gamma=gamma, radius=radius, sigma3=sigma3, sigma1=sigma1, gamma_c=gc))
