"""ctypes driver of oracle/_build/liboracle.so (vcycle_ref.c).

TEST INFRASTRUCTURE ONLY (tests/, bench.py cpu_baseline leg).  Takes a
hierarchy as plain numpy arrays -- either the Python oracle's (``from_oracle``)
or the product's exported host hierarchy (``from_levels``) -- and applies the
C restatement of the cycle on the host cores.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, '_build', 'liboracle.so')


class ocsr(C.Structure):
    _fields_ = [('n', C.c_int64), ('m', C.c_int64), ('ptr', C.c_void_p),
                ('col', C.c_void_p), ('val', C.c_void_p)]


class olevel(C.Structure):
    _fields_ = [('n', C.c_int64), ('coarsest', C.c_int),
                ('A', ocsr), ('P', ocsr), ('R', ocsr), ('W', ocsr),
                ('winv', C.c_void_p), ('Ainv', C.c_void_p),
                ('t', C.c_void_p), ('r', C.c_void_p), ('b', C.c_void_p), ('x', C.c_void_p),
                ('c', C.c_void_p), ('e', C.c_void_p), ('u', C.c_void_p)]


def _lib():
    if not os.path.exists(LIB):
        raise ImportError('oracle C library not built: make -C oracle')
    L = C.CDLL(LIB)
    L.oracle_apply.restype = C.c_int
    L.oracle_apply.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                               C.c_void_p, C.c_void_p]
    L.oracle_set_poly.restype = C.c_int
    L.oracle_set_poly.argtypes = [C.c_int, C.c_void_p]
    L.oracle_num_threads.restype = C.c_int
    L.oracle_set_threads.restype = None
    L.oracle_set_threads.argtypes = [C.c_int]
    L.oracle_pcg.restype = C.c_int
    L.oracle_pcg.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                             C.c_void_p, C.c_double, C.c_int, C.c_void_p, C.c_void_p]
    return L


class CHierarchy:
    """levels: list of dicts with keys A, P, R, WB as (indptr, indices, data,
    shape) tuples, winv, Ainv, n; params: cycle info."""

    def __init__(self, levels, wcycle=False, nu1=1, nu2=1, maxit=1, poly=None):
        self.L = _lib()
        self.keep = []
        self.poly = np.ascontiguousarray(poly if poly is not None else [], np.float64)
        self.levels = levels
        nl = len(levels)
        self.arr = (olevel * nl)()
        self.wcycle, self.nu1, self.nu2, self.maxit = int(wcycle), nu1, nu2, maxit
        for i, lv in enumerate(levels):
            o = self.arr[i]
            o.n = lv['n']
            o.coarsest = int('Ainv' in lv)
            for key in ('A', 'P', 'R', 'WB'):
                if key in lv and lv[key] is not None:
                    ip, ix, dv, shape = lv[key]
                    ip = np.ascontiguousarray(ip, np.int64)
                    ix = np.ascontiguousarray(ix, np.int32)
                    dv = np.ascontiguousarray(dv, np.float64)
                    self.keep += [ip, ix, dv]
                    s = ocsr(shape[0], shape[1], ip.ctypes.data, ix.ctypes.data, dv.ctypes.data)
                    setattr(o, 'W' if key == 'WB' else key, s)
            for key, attr in (('winv', 'winv'), ('Ainv', 'Ainv')):
                if key in lv and lv[key] is not None:
                    a = np.ascontiguousarray(lv[key], np.float64)
                    self.keep.append(a)
                    setattr(o, attr, a.ctypes.data)
            for w in ('t', 'r', 'b', 'x', 'c', 'e', 'u'):
                a = np.zeros(lv['n'])
                self.keep.append(a)
                setattr(o, w, a.ctypes.data)

    def _set_poly(self):   # the C oracle keeps the POLY weights in a global
        self.L.oracle_set_poly(len(self.poly), self.poly.ctypes.data)

    def apply(self, r):
        self._set_poly()
        r = np.ascontiguousarray(r, np.float64)
        z = np.zeros_like(r)
        rc = self.L.oracle_apply(C.cast(self.arr, C.c_void_p), len(self.levels), self.wcycle,
                                 self.nu1, self.nu2, self.maxit, r.ctypes.data, z.ctypes.data)
        if rc:
            raise RuntimeError('oracle_apply failed')
        return z

    __call__ = apply

    def pcg(self, b, tolerance=1e-8, maxiter=500):
        """cbc.block ConjGrad on level 0's A with this cycle as B (C, OpenMP):
        returns (x, residuals)."""
        self._set_poly()
        b = np.ascontiguousarray(b, np.float64)
        n = len(b)
        x = np.zeros(n)
        res = np.zeros(maxiter + 1)
        w = np.empty(4 * n)
        it = self.L.oracle_pcg(C.cast(self.arr, C.c_void_p), len(self.levels), self.wcycle, self.nu1,
                               self.nu2, self.maxit, b.ctypes.data, x.ctypes.data, float(tolerance),
                               int(maxiter), res.ctypes.data, w.ctypes.data)
        if it < 0:
            raise ValueError('Matrix is not positive')
        return x, list(res[:it + 1])

    def threads(self):
        return self.L.oracle_num_threads()

    def set_threads(self, n):
        self.L.oracle_set_threads(int(n))


def _tup(M):
    return (M.indptr, M.indices, M.data, M.shape)


def from_oracle(h):
    """CHierarchy from a Python-oracle Hierarchy (mamg_oracle.setup)."""
    levels = []
    for lv in h.levels:
        d = {'n': lv.A.shape[0], 'A': _tup(lv.A)}
        if lv.Ainv is not None:
            d['Ainv'] = lv.Ainv.ravel()
        else:
            d['P'], d['R'] = _tup(lv.P), _tup(lv.R)
            if lv.WB is not None:
                d['WB'] = _tup(lv.WB)
            else:
                d['winv'] = lv.winv
        levels.append(d)
    p = h.params
    poly = None
    if p.smoother == 'POLY':
        from mamg_oracle import poly_weights
        poly = poly_weights(p)
    return CHierarchy(levels, p.cycle_type == 'W', p.presmooth_iter, p.postsmooth_iter, p.maxit, poly)
