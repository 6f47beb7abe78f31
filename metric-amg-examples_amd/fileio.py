"""On-disk boundary of the reference's file-based pipeline.

* ``dump_system`` / ``load_system``: the ``.npy`` files of
  ``utils.dump_system`` (/root/reference/src/utils.py:304-333):
  ``A.npy`` = ``np.c_[row, col, data]`` of the monolithic COO matrix
  (float64, nnz x 3, :313-315), ``b.npy``, ``idofs.npy`` = the second block's
  dofs ``arange(W0, W0 + W1)`` (:321), ``idofs3d.npy`` = ``arange(W0)`` (:320).
* ``read_dat`` / ``dat_to_parameters``: HAZmath's ``key = value % comment``
  input file (/root/reference/src/input_metric.dat), mapped onto the
  parameter-dict keys of src/amg_parameters.py; sequential components are
  replaced by their GPU-parallel counterparts and every substitution is
  reported (parameters.to_gpu_profile).
* ``write_solution`` / ``read_solution``: ``solution.txt`` as
  src/emi_3d1d.py:148-152 reads it back -- first entry the vector size, then
  one value per line.
All loads use numpy's default ``allow_pickle=False``.
"""
from __future__ import annotations

import os
import re

import numpy as np

from . import parameters as P


def dump_system(A, b, W, folder: str) -> None:
    """Write A (scipy sparse), b, and the dof lists of a 2-block system with
    block sizes W = [dim V0, dim V1] in the reference's format."""
    import scipy.sparse as sp
    os.makedirs(folder, exist_ok=True)
    m = sp.csr_matrix(A).tocoo()
    if not np.all(np.isfinite(m.data)):
        raise ValueError('non-finite matrix entries')
    b = np.asarray(b, dtype=np.float64)
    if not np.all(np.isfinite(b)):
        raise ValueError('non-finite right-hand side')
    w0, w1 = int(W[0]), int(W[1])
    np.save(os.path.join(folder, 'A.npy'), np.c_[m.row, m.col, m.data])
    np.save(os.path.join(folder, 'b.npy'), b)
    np.save(os.path.join(folder, 'idofs.npy'), np.arange(w0, w0 + w1, dtype=np.int32))
    np.save(os.path.join(folder, 'idofs3d.npy'), np.arange(w0, dtype=np.int32))


def load_system(folder: str):
    """-> (A CSR sorted, duplicates summed; b; idofs; idofs3d)."""
    import scipy.sparse as sp
    coo = np.load(os.path.join(folder, 'A.npy'))
    if coo.ndim != 2 or coo.shape[1] != 3:
        raise ValueError('A.npy must be an nnz x 3 array [row, col, value]')
    b = np.load(os.path.join(folder, 'b.npy')).astype(np.float64)
    n = len(b)
    r, c = coo[:, 0].astype(np.int64), coo[:, 1].astype(np.int64)
    if len(r) and (r.min() < 0 or c.min() < 0 or r.max() >= n or c.max() >= n):
        raise ValueError('A.npy indices outside the size of b.npy')
    A = sp.coo_matrix((coo[:, 2], (r, c)), shape=(n, n)).tocsr()
    A.sum_duplicates()
    A.sort_indices()
    p = os.path.join(folder, 'idofs.npy')
    idofs = np.load(p).astype(np.int32) if os.path.exists(p) else None
    p = os.path.join(folder, 'idofs3d.npy')
    idofs3d = np.load(p).astype(np.int32) if os.path.exists(p) else None
    return A, b, idofs, idofs3d


_LINE = re.compile(r'^\s*([A-Za-z_][A-Za-z0-9_]*)\s*=\s*([^%;]*)')


def read_dat(path: str) -> dict:
    """HAZmath input file -> {key: value} (numbers converted, words kept)."""
    out = {}
    with open(path) as f:
        for line in f:
            if line.lstrip().startswith('%'):
                continue
            m = _LINE.match(line)
            if not m:
                continue
            key, val = m.group(1), m.group(2).strip()
            try:
                out[key] = int(val)
            except ValueError:
                try:
                    out[key] = float(val)
                except ValueError:
                    out[key] = val
    return out


_AMG_TYPE = {'UA': P.UA_AMG, 'SA': P.SA_AMG, 'MUA': P.UA_AMG, 'MSA': P.SA_AMG}
_CYCLE = {'V': P.V_CYCLE, 'W': P.W_CYCLE}
_SMOOTHER = {'JACOBI': P.SMOOTHER_JACOBI, 'L1DIAG': P.SMOOTHER_L1DIAG, 'GS': P.SMOOTHER_GS,
             'SGS': P.SMOOTHER_SGS, 'SOR': P.SMOOTHER_GS, 'SSOR': P.SMOOTHER_SGS}
_AGG = {1: P.VMB, 2: P.MIS, 3: P.MWM, 4: P.HEC, 5: P.HEM}


def dat_to_parameters(d: dict):
    """HAZmath .dat keys -> (parameter dict with src/amg_parameters.py key
    names, solver dict, substitution notes).  The solver dict carries
    linear_itsolver_type / _maxit / _tol / linear_stop_type / precond type."""
    notes = []
    prm = {}
    word = lambda k, table, default: table[str(d.get(k, default)).upper()] \
        if str(d.get(k, default)).upper() in table else None
    if 'AMG_type' in d:
        t = word('AMG_type', _AMG_TYPE, 'SA')
        if t is None:
            raise ValueError('AMG_type %r not understood' % d['AMG_type'])
        prm['AMG_type'] = t
    if 'AMG_cycle_type' in d:
        t = word('AMG_cycle_type', _CYCLE, 'V')
        if t is None:
            raise ValueError('AMG_cycle_type %r (AMLI / nonlinear AMLI / additive) is not implemented'
                             % d['AMG_cycle_type'])
        prm['cycle_type'] = t
    direct = {'AMG_levels': 'max_levels', 'AMG_maxit': 'maxit', 'AMG_relaxation': 'relaxation',
              'AMG_presmooth_iter': 'presmooth_iter', 'AMG_postsmooth_iter': 'postsmooth_iter',
              'AMG_coarse_dof': 'coarse_dof', 'AMG_coarse_solver': 'coarse_solver',
              'AMG_strong_coupled': 'strong_coupled', 'AMG_max_aggregation': 'max_aggregation',
              'AMG_amli_degree': 'amli_degree', 'AMG_Schwarz_levels': 'Schwarz_levels',
              'Schwarz_mmsize': 'Schwarz_mmsize', 'Schwarz_maxlvl': 'Schwarz_maxlvl',
              'Schwarz_type': 'Schwarz_type', 'Schwarz_blksolver': 'Schwarz_blksolver',
              'print_level': 'print_level'}
    for k, v in direct.items():
        if k in d:
            prm[v] = d[k]
    if 'AMG_smoother' in d:
        s = word('AMG_smoother', _SMOOTHER, 'GS')
        if s is None:
            raise ValueError('AMG_smoother %r not understood' % d['AMG_smoother'])
        prm['smoother'] = s
    if 'AMG_coarse_scaling' in d:
        prm['coarse_scaling'] = P.ON if str(d['AMG_coarse_scaling']).upper() == 'ON' else P.OFF
    if 'AMG_aggregation_type' in d:
        prm['aggregation_type'] = _AGG.get(int(d['AMG_aggregation_type']), P.VMB)
    maxlvl = prm.get('Schwarz_maxlvl', 1)
    mapped, n2 = P.to_gpu_profile(prm)
    # the file-based 3D-1D solve seeds the sparse 1-D dofs: HAZmath's
    # multiplicative Schwarz on their maxlvl-rings becomes the additive
    # overlapping Schwarz on the same blocks (all blocks in parallel)
    if mapped.get('Schwarz_levels', 0) >= 1 and maxlvl >= 1:
        n2 = [m for m in n2 if not m.startswith('Schwarz_maxlvl') and not m.startswith('Schwarz_type')]
        notes.append('Schwarz_type %r (multiplicative) -> SCHWARZ_ADDITIVE on the same seed + %d-ring blocks '
                     '(overlapping, parallel)' % (prm.get('Schwarz_type'), maxlvl))
        mapped['Schwarz_maxlvl'] = maxlvl
        mapped['Schwarz_type'] = P.SCHWARZ_ADDITIVE
        if prm.get('num_functions') is None:
            mapped.pop('num_functions', None)
    # the file-based 3D-1D solve seeds the 1-D dofs: its seed blocks are not
    # node-aligned, so it runs the CSR layout, where the multicolour GS
    # smoothers (node-block) do not exist; HAZmath's relaxation is an SOR
    # weight, the Jacobi smoother takes the profile's spectral weight
    if mapped.get('smoother') in (P.SMOOTHER_GS, P.SMOOTHER_SGS):
        notes.append('smoother GS/SGS -> SMOOTHER_JACOBI_RHO (seeds not node-aligned: CSR layout, '
                     'no node-block multicolour GS)')
        mapped['smoother'] = P.SMOOTHER_JACOBI_RHO
        if mapped.get('Schwarz_type') != P.SCHWARZ_ADDITIVE:
            mapped['Schwarz_type'] = P.SCHWARZ_BLOCK_JACOBI
        mapped.pop('num_functions', None)
        mapped['relaxation'] = 4.0 / 3.0
        notes.append('relaxation %s -> 4/3 (weight of the relaxation/rho Jacobi smoother)'
                     % prm.get('relaxation', 1.0))
    solver = {'type': int(d.get('linear_itsolver_type', 1)),
              'maxit': int(d.get('linear_itsolver_maxit', 500)),
              'tol': float(d.get('linear_itsolver_tol', 1e-6)),
              'stop_type': int(d.get('linear_stop_type', 1)),
              'precond_type': int(d.get('linear_precond_type', 16))}
    if solver['type'] != 1:
        raise ValueError('linear_itsolver_type %d: only 1 (CG) is implemented' % solver['type'])
    if solver['stop_type'] not in (1, 2):
        raise ValueError('linear_stop_type %d: only 1 (||r||/||b||) and 2 (||r||_B/||b||_B)'
                         % solver['stop_type'])
    return mapped, solver, notes + n2


def write_solution(path: str, x: np.ndarray) -> None:
    """solution.txt: the size, then one value per line (src/emi_3d1d.py:148-152)."""
    x = np.asarray(x, dtype=np.float64)
    with open(path, 'w') as f:
        f.write('%d\n' % len(x))
        np.savetxt(f, x, fmt='%.17e')


def read_solution(path: str) -> np.ndarray:
    sol = np.loadtxt(path)
    size = int(sol[0])
    return sol[1:size + 1]
